"""Build protobuf message classes and gRPC service bindings from Python.

The image has grpcio and protobuf but no ``protoc`` / ``grpc_tools``, so the
wire contracts (the arena's ``inference`` package and the KServe-v2 predict
protocol) are declared here as ``FileDescriptorProto`` objects and turned
into message classes at import time.  The reference instead generates and
git-ignores ``*_pb2.py`` stubs (src/shared/proto/__init__.py:27-73,
scripts/generate_proto.py:61-136); the wire format is identical.

Small DSL::

    f = ProtoFile("inference/x.proto", "inference")
    f.message("Box", [("x1", 1, "float"), ("ids", 2, "int32", "repeated")])
    f.service("Svc", [("Get", "Box", "Box")])
    mods = f.build()     # namespace with message classes + services
"""
from __future__ import annotations

from dataclasses import dataclass, field
from types import SimpleNamespace

from google.protobuf import descriptor_pb2, descriptor_pool, message_factory

_T = descriptor_pb2.FieldDescriptorProto
SCALARS = {
    "double": _T.TYPE_DOUBLE, "float": _T.TYPE_FLOAT, "int64": _T.TYPE_INT64, "uint64": _T.TYPE_UINT64,
    "int32": _T.TYPE_INT32, "uint32": _T.TYPE_UINT32, "bool": _T.TYPE_BOOL, "string": _T.TYPE_STRING,
    "bytes": _T.TYPE_BYTES,
}
LABELS = {"optional": _T.LABEL_OPTIONAL, "repeated": _T.LABEL_REPEATED}

# One private pool for every arena contract, so cross-file references resolve.
POOL = descriptor_pool.DescriptorPool()


@dataclass
class _Msg:
    name: str
    fields: list
    nested: list = field(default_factory=list)
    enums: list = field(default_factory=list)
    oneofs: dict = field(default_factory=dict)  # field name -> oneof name


class ProtoFile:
    def __init__(self, name: str, package: str, deps: list[str] | None = None):
        self.fp = descriptor_pb2.FileDescriptorProto(name=name, package=package, syntax="proto3")
        self.fp.dependency.extend(deps or [])
        self.package = package
        self._services: list[str] = []

    # ------------------------------------------------------------------ messages
    def _fill(self, mp: descriptor_pb2.DescriptorProto, m: _Msg, scope: str) -> None:
        mp.name = m.name
        full = f"{scope}.{m.name}"
        for e_name, values in m.enums:
            ep = mp.enum_type.add(name=e_name)
            for v_name, num in values:
                ep.value.add(name=v_name, number=num)
        for sub in m.nested:
            self._fill(mp.nested_type.add(), sub, full)
        oneof_index: dict[str, int] = {}
        for spec in m.fields:
            name, num, typ = spec[:3]
            label = spec[3] if len(spec) > 3 else "optional"
            fp = mp.field.add(name=name, number=num, json_name=_json_name(name))
            if typ.startswith("map<"):
                k, v = typ[4:-1].split(",")
                entry = _Msg(_entry_name(name), [("key", 1, k.strip()), ("value", 2, v.strip())])
                ep = mp.nested_type.add()
                self._fill(ep, entry, full)
                ep.options.map_entry = True
                fp.label = _T.LABEL_REPEATED
                fp.type = _T.TYPE_MESSAGE
                fp.type_name = f"{full}.{entry.name}"
                continue
            fp.label = LABELS[label]
            if typ in SCALARS:
                fp.type = SCALARS[typ]
            elif typ.startswith("enum:"):
                fp.type = _T.TYPE_ENUM
                fp.type_name = self._resolve(typ[5:], full)
            else:
                fp.type = _T.TYPE_MESSAGE
                fp.type_name = self._resolve(typ, full)
            if name in m.oneofs:
                o = m.oneofs[name]
                if o not in oneof_index:
                    oneof_index[o] = len(mp.oneof_decl)
                    mp.oneof_decl.add(name=o)
                fp.oneof_index = oneof_index[o]

    def _resolve(self, typ: str, scope: str) -> str:
        if typ.startswith("."):
            return typ
        if "." in typ:  # Outer.Inner relative to the package
            return f".{self.package}.{typ}"
        return f".{self.package}.{typ}"

    def message(self, name: str, fields: list, nested: list | None = None, enums: list | None = None,
                oneofs: dict | None = None) -> _Msg:
        m = _Msg(name, fields, nested or [], enums or [], oneofs or {})
        self._fill(self.fp.message_type.add(), m, f".{self.package}")
        return m

    @staticmethod
    def nested(name: str, fields: list, nested: list | None = None, enums: list | None = None,
               oneofs: dict | None = None) -> _Msg:
        return _Msg(name, fields, nested or [], enums or [], oneofs or {})

    # ------------------------------------------------------------------ services
    def service(self, name: str, methods: list[tuple[str, str, str]]) -> None:
        sp = self.fp.service.add(name=name)
        for m, req, resp in methods:
            sp.method.add(name=m, input_type=self._resolve(req, ""), output_type=self._resolve(resp, ""))
        self._services.append(name)

    def build(self) -> SimpleNamespace:
        fd = POOL.Add(self.fp)
        fd = POOL.FindFileByName(self.fp.name)
        ns = SimpleNamespace()
        for name, desc in fd.message_types_by_name.items():
            setattr(ns, name, message_factory.GetMessageClass(desc))
        ns.services = {}
        for name, sd in fd.services_by_name.items():
            ns.services[name] = Service(sd)
        ns.DESCRIPTOR = fd
        return ns


def _json_name(name: str) -> str:
    parts = name.split("_")
    return parts[0] + "".join(p[:1].upper() + p[1:] for p in parts[1:])


def _entry_name(field_name: str) -> str:
    return "".join(p[:1].upper() + p[1:] for p in field_name.split("_")) + "Entry"


class Service:
    """gRPC bindings for one service descriptor: server handler + client stubs."""

    def __init__(self, sd):
        self.sd = sd
        self.full_name = sd.full_name
        self.methods = {}
        for m in sd.methods:
            self.methods[m.name] = (message_factory.GetMessageClass(m.input_type),
                                    message_factory.GetMessageClass(m.output_type))

    def path(self, method: str) -> str:
        return f"/{self.full_name}/{method}"

    def handler(self, impl) -> "object":
        """Generic handler routing each method to ``impl.<Method>(request, context)``
        (sync or ``async def`` — grpc picks the matching server flavour)."""
        import grpc

        table = {}
        for name, (req, resp) in self.methods.items():
            fn = getattr(impl, name, None)
            if fn is None:
                continue
            table[name] = grpc.unary_unary_rpc_method_handler(
                fn, request_deserializer=req.FromString, response_serializer=resp.SerializeToString)
        return grpc.method_handlers_generic_handler(self.full_name, table)

    def stub(self, channel) -> SimpleNamespace:
        """Client stub: ``stub.Method(request, timeout=...)`` for a sync or aio channel."""
        ns = SimpleNamespace()
        for name, (req, resp) in self.methods.items():
            setattr(ns, name, channel.unary_unary(self.path(name), request_serializer=req.SerializeToString,
                                                  response_deserializer=resp.FromString))
        return ns
