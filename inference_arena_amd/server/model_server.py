"""Arena model server front-ends: KServe-v2 gRPC (:8001), HTTP/REST (:8000),
Prometheus metrics (:8002) — the ports and protocol of the Triton server the
reference deploys (architectures/triton/docker-compose.yml:79-147; client
calls in architectures/triton/gateway/app/triton_client.py:39-179).

gRPC  inference.GRPCInferenceService: ServerLive, ServerReady, ModelReady,
      ServerMetadata, ModelMetadata, ModelInfer (raw_input_contents or typed
      contents; BYTES tensors length-prefixed), RepositoryIndex,
      ModelStatistics.  Errors: NOT_FOUND / INVALID_ARGUMENT / UNAVAILABLE /
      INTERNAL status codes.
HTTP  GET /v2, /v2/health/live, /v2/health/ready, /v2/models/{m}[/versions/{v}],
      /v2/models/{m}[/versions/{v}]/ready, POST /v2/models/{m}[/versions/{v}]/infer
      (JSON tensors, plus the binary-tensor extension:
      ``Inference-Header-Content-Length``), POST /v2/repository/index,
      GET /v2/models/{m}/stats.
Metrics nv_inference_* counters/durations per model (Triton metric names, so
      existing dashboards keep working) plus arena batcher gauges.

Run: ``python -m inference_arena_amd.server.model_server --model-repository model_repository``.
"""
from __future__ import annotations

import argparse
import asyncio
import json
import logging
import os

import grpc
import numpy as np
from fastapi import FastAPI, HTTPException, Request
from fastapi.responses import JSONResponse, Response

from ..proto import kserve as kv
from ..utils.logging import setup_logging
from .modelserver_core import InferError, ModelServer

log = logging.getLogger("arena.modelserver")
MAX_MESSAGE = 64 * 1024 * 1024
GRPC_OPTIONS = [("grpc.max_send_message_length", MAX_MESSAGE), ("grpc.max_receive_message_length", MAX_MESSAGE)]
_GRPC_CODES = {"NOT_FOUND": grpc.StatusCode.NOT_FOUND, "INVALID_ARGUMENT": grpc.StatusCode.INVALID_ARGUMENT,
               "UNAVAILABLE": grpc.StatusCode.UNAVAILABLE}


# ----------------------------------------------------------------------------- gRPC
class KServeServicer:
    def __init__(self, server: ModelServer):
        self.s = server

    async def ServerLive(self, req, ctx):
        return kv.ServerLiveResponse(live=self.s.live())

    async def ServerReady(self, req, ctx):
        return kv.ServerReadyResponse(ready=self.s.ready())

    async def ModelReady(self, req, ctx):
        m = self.s.models.get(req.name)
        return kv.ModelReadyResponse(ready=bool(m and m.ready))

    async def ServerMetadata(self, req, ctx):
        return kv.ServerMetadataResponse(name=self.s.name, version=self.s.version, extensions=self.s.extensions)

    async def ModelMetadata(self, req, ctx):
        try:
            md = self.s.get(req.name, req.version).metadata()
        except InferError as e:
            await ctx.abort(_GRPC_CODES.get(e.code, grpc.StatusCode.INVALID_ARGUMENT), str(e))
        r = kv.ModelMetadataResponse(name=md["name"], versions=md["versions"], platform=md["platform"])
        for src, dst in ((md["inputs"], r.inputs), (md["outputs"], r.outputs)):
            for t in src:
                dst.add(name=t["name"], datatype=t["datatype"], shape=t["shape"])
        return r

    async def ModelInfer(self, req, ctx):
        try:
            inputs = {t.name: kv.decode_input(req, i) for i, t in enumerate(req.inputs)}
        except ValueError as e:
            await ctx.abort(grpc.StatusCode.INVALID_ARGUMENT, str(e))
        try:
            out = await self.s.infer(req.model_name, inputs, [o.name for o in req.outputs] or None,
                                     req.model_version)
        except InferError as e:
            await ctx.abort(_GRPC_CODES.get(e.code, grpc.StatusCode.INVALID_ARGUMENT), str(e))
        except Exception as e:  # noqa: BLE001
            log.error(f"ModelInfer failed: {e}")
            await ctx.abort(grpc.StatusCode.INTERNAL, str(e))
        m = self.s.models[req.model_name]
        resp = kv.ModelInferResponse(model_name=req.model_name, model_version=m.version, id=req.id)
        for name, arr in out.items():
            kv.encode_output(resp, name, arr)
        return resp

    async def RepositoryIndex(self, req, ctx):
        r = kv.RepositoryIndexResponse()
        for e in self.s.index():
            if req.ready and e["state"] != "READY":
                continue
            r.models.add(**e)
        return r

    async def ModelStatistics(self, req, ctx):
        r = kv.ModelStatisticsResponse()
        names = [req.name] if req.name else list(self.s.models)
        for n in names:
            m = self.s.models.get(n)
            if m is None:
                await ctx.abort(grpc.StatusCode.NOT_FOUND, f"unknown model '{n}'")
            st = m.stats
            r.model_stats.add(name=n, version=m.version, last_inference=st.last_inference_ms,
                              inference_count=st.inference_count, execution_count=st.execution_count)
        return r


async def start_grpc(server: ModelServer, host: str, port: int):
    g = grpc.aio.server(options=GRPC_OPTIONS)
    g.add_generic_rpc_handlers((kv.GRPCInferenceService.handler(KServeServicer(server)),))
    bound = g.add_insecure_port(f"{host}:{port}")
    await g.start()
    return g, bound


# ----------------------------------------------------------------------------- HTTP
_NP = {k: v for k, v in kv.DTYPES.items()}


def _json_input(t: dict, binary: bytes | None) -> np.ndarray:
    dt = t.get("datatype", "")
    shape = [int(s) for s in t.get("shape", [])]
    if dt == "BYTES":
        items = kv.deserialize_bytes(binary) if binary is not None else \
            [x.encode() if isinstance(x, str) else bytes(x) for x in np.ravel(t.get("data", []))]
        a = np.empty(len(items), dtype=object)
        a[:] = items
        return a.reshape(shape)
    if dt not in _NP:
        raise InferError(f"unsupported datatype '{dt}'")
    if binary is not None:
        a = np.frombuffer(binary, dtype=_NP[dt])
    else:
        a = np.asarray(t.get("data", []), dtype=_NP[dt]).ravel()
    if a.size != int(np.prod(shape)):
        raise InferError(f"input '{t.get('name')}': {a.size} elements for shape {shape}")
    return a.reshape(shape)


def create_http_app(server: ModelServer) -> FastAPI:
    app = FastAPI(title="Arena model server (KServe v2)", version=server.version)

    def _err(e: InferError):
        return JSONResponse({"error": str(e)}, status_code=404 if e.code == "NOT_FOUND" else 400)

    @app.get("/v2")
    async def server_meta():
        return {"name": server.name, "version": server.version, "extensions": server.extensions}

    @app.get("/v2/health/live")
    async def live():
        return Response(status_code=200 if server.live() else 400)

    @app.get("/v2/health/ready")
    async def ready():
        return Response(status_code=200 if server.ready() else 400)

    @app.get("/v2/models/{name}")
    @app.get("/v2/models/{name}/versions/{version}")
    async def model_meta(name: str, version: str = ""):
        try:
            return server.get(name, version).metadata()
        except InferError as e:
            return _err(e)

    @app.get("/v2/models/{name}/ready")
    @app.get("/v2/models/{name}/versions/{version}/ready")
    async def model_ready(name: str, version: str = ""):
        m = server.models.get(name)
        return Response(status_code=200 if m is not None and m.ready else 400)

    @app.get("/v2/models/{name}/config")
    async def model_config(name: str):
        from google.protobuf import json_format

        try:
            return json_format.MessageToDict(server.get(name).config, preserving_proto_field_name=True)
        except InferError as e:
            return _err(e)

    @app.get("/v2/models/{name}/stats")
    @app.get("/v2/models/stats")
    async def model_stats(name: str = ""):
        out = []
        for n, m in server.models.items():
            if name and n != name:
                continue
            st = m.stats
            out.append({"name": n, "version": m.version, "last_inference": st.last_inference_ms,
                        "inference_count": st.inference_count, "execution_count": st.execution_count,
                        "inference_stats": {"success": {"count": st.success, "ns": int(st.request_us * 1e3)},
                                            "fail": {"count": st.failure},
                                            "queue": {"ns": int(st.queue_us * 1e3)},
                                            "compute_infer": {"ns": int(st.compute_us * 1e3)}}})
        if name and not out:
            return JSONResponse({"error": f"unknown model '{name}'"}, status_code=404)
        return {"model_stats": out}

    @app.post("/v2/repository/index")
    async def repo_index():
        return server.index()

    @app.post("/v2/models/{name}/infer")
    @app.post("/v2/models/{name}/versions/{version}/infer")
    async def infer(name: str, request: Request, version: str = ""):
        body = await request.body()
        hlen = request.headers.get("inference-header-content-length")
        try:
            if hlen is not None:
                n = int(hlen)
                header = json.loads(body[:n])
                blob = body[n:]
            else:
                header = json.loads(body or b"{}")
                blob = b""
            inputs, off = {}, 0
            for t in header.get("inputs", []):
                size = (t.get("parameters") or {}).get("binary_data_size")
                binary = None
                if size is not None:
                    binary = blob[off:off + int(size)]
                    off += int(size)
                inputs[t["name"]] = _json_input(t, binary)
            req_out = header.get("outputs") or []
            names = [o["name"] for o in req_out] or None
            want_bin = {o["name"] for o in req_out if (o.get("parameters") or {}).get("binary_data")}
            if (header.get("parameters") or {}).get("binary_data_output"):
                want_bin = {"*"}
            out = await server.infer(name, inputs, names, version)
        except InferError as e:
            return _err(e)
        except (ValueError, KeyError, json.JSONDecodeError) as e:
            return JSONResponse({"error": f"malformed request: {e}"}, status_code=400)
        except Exception as e:  # noqa: BLE001
            raise HTTPException(status_code=500, detail=str(e)) from e
        m = server.models[name]
        outs, blobs = [], []
        for k, arr in out.items():
            d = {"name": k, "datatype": kv.datatype_of(arr), "shape": list(arr.shape)}
            if k in want_bin or "*" in want_bin:
                b = np.ascontiguousarray(arr).tobytes()
                d["parameters"] = {"binary_data_size": len(b)}
                blobs.append(b)
            else:
                d["data"] = arr.ravel().tolist()
            outs.append(d)
        js = json.dumps({"model_name": name, "model_version": m.version, "id": header.get("id", ""),
                         "outputs": outs}).encode()
        if blobs:
            return Response(js + b"".join(blobs), media_type="application/octet-stream",
                            headers={"Inference-Header-Content-Length": str(len(js))})
        return Response(js, media_type="application/json")

    return app


# ----------------------------------------------------------------------------- metrics
def render_metrics(server: ModelServer) -> bytes:
    from prometheus_client import CollectorRegistry, Counter, Gauge, generate_latest

    reg = CollectorRegistry()
    lab = ["model", "version"]
    succ = Counter("nv_inference_request_success", "Successful requests", lab, registry=reg)
    fail = Counter("nv_inference_request_failure", "Failed requests", lab, registry=reg)
    cnt = Counter("nv_inference_count", "Inferences (batch items)", lab, registry=reg)
    exe = Counter("nv_inference_exec_count", "Executions", lab, registry=reg)
    dur = Counter("nv_inference_request_duration_us", "Cumulative request time", lab, registry=reg)
    que = Counter("nv_inference_queue_duration_us", "Cumulative queue time", lab, registry=reg)
    cmp_ = Counter("nv_inference_compute_infer_duration_us", "Cumulative compute time", lab, registry=reg)
    qd = Gauge("arena_batcher_queue_depth", "Requests waiting in the dynamic batcher", lab, registry=reg)
    mb = Gauge("arena_batcher_mean_batch", "Mean executed batch size", lab, registry=reg)
    for n, m in server.models.items():
        st = m.stats
        lv = (n, m.version)
        succ.labels(*lv).inc(st.success)
        fail.labels(*lv).inc(st.failure)
        cnt.labels(*lv).inc(st.inference_count)
        exe.labels(*lv).inc(st.execution_count)
        dur.labels(*lv).inc(st.request_us)
        que.labels(*lv).inc(st.queue_us)
        cmp_.labels(*lv).inc(st.compute_us)
        b = getattr(m, "batcher", None) or getattr(getattr(m, "backend", None), "batcher", None)
        if b is not None:
            s = b.stats()
            qd.labels(*lv).set(s.get("queue_depth", 0))
            mb.labels(*lv).set(s.get("mean_batch", 0))
    return generate_latest(reg)


def create_metrics_app(server: ModelServer) -> FastAPI:
    app = FastAPI(title="Arena model server metrics")

    @app.get("/metrics")
    async def metrics():
        return Response(render_metrics(server), media_type="text/plain; version=0.0.4")

    return app


# ----------------------------------------------------------------------------- main
def start_native_kserve(server: ModelServer, host_ip: str, port: int, model: str = "arena_pipeline",
                        host: dict | None = None):
    """The ensemble's hot path without Python: a native HTTP front end (csrc/runtime/http_front.h with
    ``kserve_model``) on ``port`` serving KServe-v2 REST infer requests for ``model`` (binary tensor extension)
    straight into the ensemble's native dynamic batcher, with the split JPEG decoder on C++ threads — the endpoint
    the native gateway (server/native_gateway.py) forwards to.  None when off (port 0), on CPU, or when the model
    is not a GPU-batched pipeline."""
    if port <= 0 or server.device not in ("gpu", "fake"):
        return None
    m = server.models.get(model)
    backend = getattr(m, "backend", None)
    batcher = getattr(getattr(backend, "batcher", None), "_b", None)
    if batcher is None:
        log.warning(f"native KServe endpoint: model {model} has no native batcher; endpoint off")
        return None
    from ..labels import load_labels
    from .native_front import NativeFrontEnd

    plan = (host or {}).get("plan") or {"http_io": int(os.environ.get("ARENA_HTTP_THREADS", "4")),
                                         "decode_threads": int(os.environ.get("ARENA_DECODE_THREADS", "8"))}
    fe = NativeFrontEnd(batcher, load_labels(None), port=port, host=host_ip, arch="triton",
                        io_threads=plan["http_io"], decode_threads=plan["decode_threads"],
                        decode_procs=int(os.environ.get("ARENA_DECODE_PROCS", "1") or 1), kserve_model=model,
                        gpu=str((host or {}).get("gpu", 0)), jpeg_device=server.device == "gpu")
    if host:
        from ..parallel.affinity import rank_info_metrics

        fe.extra_metrics = rank_info_metrics(dict(host, plan=plan), "triton")
    return fe


async def serve(args) -> None:
    """Run until SIGINT / SIGTERM, then shut down like the reference classification service
    (architectures/microservices/classification/app/main.py:86-104): stop accepting, give in-flight RPCs a 5 s
    grace, close the backends (batchers, decode processes, shared memory) and return normally — no traceback."""
    import contextlib
    import signal

    import uvicorn

    class _Server(uvicorn.Server):
        @contextlib.contextmanager
        def capture_signals(self):  # the process-wide handlers below own SIGINT / SIGTERM
            yield

    setup_logging(args.log_level)
    from .replica import _socket

    # one model-server process per GPU (scripts/start_arena.py --arch triton): ARENA_LOCAL_WORLD processes on the
    # node, this one serving GPU args.gpu; it pins itself to that GPU's CPU share and sizes its threads for it
    world = int(os.environ.get("ARENA_LOCAL_WORLD", "1") or 1)
    host = None
    if world > 1 or os.environ.get("ARENA_RANK_PLAN") == "1":
        from ..parallel.affinity import rank_host_setup

        host = rank_host_setup(args.gpu, world)
        log.info(f"model server rank: gpu {args.gpu} of {world}, cpus {host['cpus']}, usable {host['usable_cpus']}, "
                 f"host plan {host['plan']}")
    server = ModelServer(args.model_repository, device=args.device, gpu=args.gpu)
    stop = asyncio.Event()
    loop = asyncio.get_running_loop()
    for sig in (signal.SIGINT, signal.SIGTERM):
        loop.add_signal_handler(sig, stop.set)
    # every port is opened with SO_REUSEPORT (gRPC's default), so several server processes on
    # one GPU can share :8000/:8001/:8002 and the kernel spreads connections over them
    g, _ = await start_grpc(server, args.host, args.grpc_port)
    apps = [(create_http_app(server), args.http_port), (create_metrics_app(server), args.metrics_port)]
    servers, socks = [], []
    for app, port in apps:
        socks.append(_socket(args.host, port, reuse_port=True))
        servers.append(_Server(uvicorn.Config(app, log_level="warning", access_log=False)))
    native_fe = start_native_kserve(server, args.host, args.native_http_port, host=host)
    log.info(f"model server ready: grpc {args.grpc_port} http {args.http_port} metrics {args.metrics_port}"
             + (f" native-kserve {native_fe.port}" if native_fe else ""))
    tasks = [asyncio.create_task(s.serve(sockets=[k])) for s, k in zip(servers, socks)]
    try:
        await stop.wait()
        log.info("shutting down: draining in-flight requests (5 s grace)")
    finally:
        for s in servers:
            s.should_exit = True
        await g.stop(grace=5)
        await asyncio.wait(tasks, timeout=10)
        if native_fe is not None:
            native_fe.close()
        server.close()
        log.info("model server stopped")


def main(argv=None) -> None:
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--model-repository", default=os.environ.get("MODELS_DIR", "model_repository"))
    ap.add_argument("--host", default="0.0.0.0")
    ap.add_argument("--http-port", type=int, default=8000)
    ap.add_argument("--grpc-port", type=int, default=8001)
    ap.add_argument("--metrics-port", type=int, default=8002)
    ap.add_argument("--native-http-port", type=int, default=int(os.environ.get("ARENA_KSERVE_NATIVE_PORT", "8004")),
                    help="native KServe-v2 REST endpoint of the arena_pipeline ensemble (0: off)")
    ap.add_argument("--device", default=os.environ.get("ARENA_DEVICE", "gpu"), choices=["gpu", "cpu", "fake"])
    ap.add_argument("--gpu", type=int, default=int(os.environ.get("ARENA_GPU", "0")))
    ap.add_argument("--log-level", default=os.environ.get("LOG_LEVEL", "INFO"))
    from .decode_pool import prestart

    prestart()  # decode-worker fork server before the engines touch the GPU (the native endpoint's PIL fallback)
    asyncio.run(serve(ap.parse_args(argv)))


if __name__ == "__main__":
    main()
