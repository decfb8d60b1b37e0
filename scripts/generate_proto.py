#!/usr/bin/env python3
"""Write .proto text for the contracts that are defined in code (for external clients).

The reference keeps inference.proto as the source and generates Python stubs
(scripts/generate_proto.py:61-136); here the descriptors built by
inference_arena_amd.proto are the source and this script renders them back
to proto3 text: arena/inference.proto, arena/kserve_v2.proto and
arena/model_config.proto.
"""
from __future__ import annotations

import argparse
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

_TYPES = {1: "double", 2: "float", 3: "int64", 4: "uint64", 5: "int32", 8: "bool", 9: "string", 12: "bytes",
          13: "uint32"}


def render(fd) -> str:
    from google.protobuf import descriptor_pb2

    fp = descriptor_pb2.FileDescriptorProto()
    fd.CopyToProto(fp)
    out = [f'syntax = "proto3";', f"package {fp.package};", ""]

    def tname(f, scope):
        if f.type in (11, 14):
            n = f.type_name.lstrip(".")
            return n[len(fp.package) + 1:] if n.startswith(fp.package + ".") else n
        return _TYPES[f.type]

    def msg(m, ind, scope):
        pad = "  " * ind
        out.append(f"{pad}message {m.name} {{")
        maps = {n.name: n for n in m.nested_type if n.options.map_entry}
        for e in m.enum_type:
            out.append(f"{pad}  enum {e.name} {{")
            for v in e.value:
                out.append(f"{pad}    {v.name} = {v.number};")
            out.append(f"{pad}  }}")
        for n in m.nested_type:
            if not n.options.map_entry:
                msg(n, ind + 1, scope + "." + m.name)
        oneofs = {}
        for f in m.field:
            if f.HasField("oneof_index"):
                oneofs.setdefault(f.oneof_index, []).append(f)
                continue
            entry = f.type_name.rsplit(".", 1)[-1]
            if f.label == 3 and entry in maps:
                k, v = maps[entry].field
                out.append(f"{pad}  map<{tname(k, scope)}, {tname(v, scope)}> {f.name} = {f.number};")
            else:
                rep = "repeated " if f.label == 3 else ""
                out.append(f"{pad}  {rep}{tname(f, scope)} {f.name} = {f.number};")
        for idx, fs in oneofs.items():
            out.append(f"{pad}  oneof {m.oneof_decl[idx].name} {{")
            for f in fs:
                out.append(f"{pad}    {tname(f, scope)} {f.name} = {f.number};")
            out.append(f"{pad}  }}")
        out.append(f"{pad}}}")

    for m in fp.message_type:
        msg(m, 0, fp.package)
        out.append("")
    for s in fp.service:
        out.append(f"service {s.name} {{")
        for meth in s.method:
            i = meth.input_type.rsplit(".", 1)[-1]
            o = meth.output_type.rsplit(".", 1)[-1]
            out.append(f"  rpc {meth.name}({i}) returns ({o});")
        out.append("}")
        out.append("")
    return "\n".join(out)


def main(argv=None) -> int:
    from inference_arena_amd.proto import inference_api, kserve
    from inference_arena_amd.repository import model_config

    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--out", default="proto")
    a = ap.parse_args(argv)
    out = Path(a.out)
    out.mkdir(parents=True, exist_ok=True)
    for name, mod in (("inference.proto", inference_api), ("kserve_v2.proto", kserve),
                      ("model_config.proto", model_config)):
        (out / name).write_text(render(mod.pb.DESCRIPTOR) + "\n")
        print(f"wrote {out / name}")
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
