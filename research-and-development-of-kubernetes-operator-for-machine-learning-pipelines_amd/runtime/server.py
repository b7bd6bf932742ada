"""The predictor container: V2 ("kfserving") inference protocol server (G6).

Endpoints (the SeldonDeployment's ``protocol: kfserving`` / Open Inference Protocol):
  GET  /v2/health/live | /v2/health/ready | /v2 | /v2/models/{m} | /v2/models/{m}/ready
  POST /v2/models/{m}/infer             tensors in / tensors out (sklearn or LLM)
  POST /v2/models/{m}/generate          {"text_input" | "input_ids", "parameters": {...}}
  POST /v2/models/{m}/generate_stream   server-sent events, one per token
  POST /api/v1.0/feedback               Seldon feedback (counted as service="feedback")
  GET  /metrics                         Prometheus exposition (runtime/metrics.py)

Every request is timed into the Seldon-executor histograms with its HTTP
code, which is what the operator's canary gate queries.

``python -m mlopamd.runtime.server --runtime mlop-llm --architecture llama3-8b``
starts it; configuration also comes from the env the SeldonDeployment sets
(MLOP_RUNTIME, MLOP_MODEL_URI, MLOP_ARCHITECTURE, MLOP_ENGINE_*, MLOP_DTYPE).  A model URI that
resolves to a local Hugging Face checkpoint (models/loader.py) is served with its weights and
``tokenizer.json``; otherwise the architecture is random-initialised (the benchmark setup).
Fault injection for canary tests: MLOP_INJECT_LATENCY_S, MLOP_INJECT_ERROR_RATE,
MLOP_INJECT_START_ERROR (fail at start-up, e.g. a GPU OOM message), MLOP_INJECT_CRASH_AFTER_S
(exit with status 139 after serving that long).
"""
from __future__ import annotations

import argparse
import asyncio
import json
import os
import random
import time

import numpy as np

# start-up phases of this predictor process, seconds since the OS created it (GET /v2/debug/startup;
# bench.py's fresh-process CR -> ready probe reports them): what the 2 s of a cold start go to
STARTUP: dict = {}


def _since_process_start() -> float:
    """Seconds since the launcher started this process (MLOP_LAUNCH_EPOCH, its wall clock right
    before the spawn: exact on one host), else since the kernel's process creation time (psutil:
    clock-tick resolution on an integer-second boot time, so only differences are meaningful)."""
    t0 = os.environ.get("MLOP_LAUNCH_EPOCH")
    if t0:
        return round(time.time() - float(t0), 3)
    try:
        import psutil

        return round(time.time() - psutil.Process().create_time(), 3)
    except Exception:  # noqa: BLE001
        return -1.0


STARTUP["server_module_imported_s"] = _since_process_start()
if os.environ.get("MLOP_LAUNCHER_INFO"):  # this rank's pod launcher (rank_launcher.py) about itself
    STARTUP["launcher"] = json.loads(os.environ["MLOP_LAUNCHER_INFO"])

if __name__ == "__main__":
    import sys as _sys

    # one module object whether reached as __main__ or as a package import (tp_worker /
    # ep_serving import make_app from here): one STARTUP dict, one set of globals
    _sys.modules.setdefault(f"{__package__}.server", _sys.modules[__name__])

    # a multi-rank pod's container process is a LAUNCHER: decided from argv / env alone, before
    # torch is imported and before any HIP call, and it never comes back here (rank_launcher.py)
    from .rank_launcher import launch_ranks as _launch_ranks, launcher_degree as _launcher_degree

    _n_ranks = _launcher_degree(_sys.argv[1:])
    if _n_ranks > 1:
        raise SystemExit(_launch_ranks(_n_ranks, _sys.argv[1:]))


def _warm_hip() -> None:
    """Initialise the HIP runtime and this rank's device context on a helper thread WHILE torch
    imports (~1.4 s of Python and dlopen): the C calls release the GIL, and torch's own first
    device call then finds the runtime up (first allocation 0.15-0.35 s -> ~0.1 s,
    scripts/probe_startup.py).  Off for CPU predictors and with MLOP_HIP_WARMUP=0."""
    import ctypes
    import importlib.util

    try:
        # torch's OWN copy of the runtime (its lib/ directory, found without importing torch): a
        # bare "libamdhip64.so" could resolve to the system ROCm copy, and a second HIP runtime
        # in the process would not be the one torch and _C.so launch on
        spec = importlib.util.find_spec("torch")
        if spec is None or not spec.origin:
            return
        lib = ctypes.CDLL(os.path.join(os.path.dirname(spec.origin), "lib", "libamdhip64.so"))
        if lib.hipInit(0) == 0 and lib.hipSetDevice(int(os.environ.get("LOCAL_RANK", "0"))) == 0:
            lib.hipFree(ctypes.c_void_p(0))  # creates the device context
        STARTUP["hip_warm_s"] = _since_process_start()
    except OSError:
        pass


def start_hip_warmup() -> bool:
    """Start ``_warm_hip`` on a daemon thread in a process that will itself run a GPU engine:
    the predictor's ``__main__`` once it is known not to be a multi-rank launcher (above), never
    on import as a library.  Off for CPU / sklearn predictors and with MLOP_HIP_WARMUP=0."""
    if (os.environ.get("MLOP_DEVICE", "cuda") == "cpu" or os.environ.get("MLOP_HIP_WARMUP", "1") == "0"
            or os.environ.get("MLOP_RUNTIME", "mlop-llm") in ("mlop-sklearn", "sklearn")):
        return False
    import threading

    from . import rank_launcher

    rank_launcher.WARMUP_STARTED = True
    STARTUP["hip_warmup_started"] = True
    threading.Thread(target=_warm_hip, name="hip-warmup", daemon=True).start()
    return True


if __name__ == "__main__":
    start_hip_warmup()

from .sampler import SamplingParams  # noqa: E402 (imports torch: timed below)

STARTUP["torch_imported_s"] = _since_process_start()

_DT = {"FP32": np.float32, "FP64": np.float64, "INT64": np.int64, "INT32": np.int32, "FP16": np.float16,
       "BOOL": np.bool_, "UINT8": np.uint8}
_DT_NAME = {np.dtype(v): k for k, v in _DT.items()}


def _params(p: dict) -> SamplingParams:
    return SamplingParams(max_tokens=int(p.get("max_tokens", 64)), temperature=float(p.get("temperature", 0.0)),
                          top_k=int(p.get("top_k", 0)), top_p=float(p.get("top_p", 1.0)),
                          ignore_eos=bool(p.get("ignore_eos", False)),
                          stop_token_ids=list(p.get("stop_token_ids", [])),
                          seed=None if p.get("seed") is None else int(p["seed"]))


def make_app(backend, metrics, version: str = "1", inject_latency_s: float | None = None,
             inject_error_rate: float | None = None):
    from aiohttp import web

    lat = float(os.environ.get("MLOP_INJECT_LATENCY_S", inject_latency_s or 0.0))
    err_rate = float(os.environ.get("MLOP_INJECT_ERROR_RATE", inject_error_rate or 0.0))
    state = {"ready": getattr(backend, "ready", True)}

    @web.middleware
    async def timing(request, handler):
        t0 = time.perf_counter()
        service = "feedback" if request.path.endswith("/feedback") else (
            "generate" if "generate" in request.path else "predictions")
        code = 500
        try:
            if request.method == "POST" and not request.path.endswith("/feedback"):
                if lat:
                    await asyncio.sleep(lat)
                if err_rate and random.random() < err_rate:
                    raise web.HTTPInternalServerError(text="injected failure")
            try:
                resp = await handler(request)
            except ValueError as e:  # a request the engine refuses (engine.check_request): the client's error
                raise web.HTTPBadRequest(text=str(e)) from None
            code = resp.status
            return resp
        except web.HTTPException as e:
            code = e.status
            raise
        finally:
            if request.method == "POST" and metrics is not None:
                metrics.observe_request(time.perf_counter() - t0, code=code, service=service)

    app = web.Application(middlewares=[timing], client_max_size=64 * 2**20)

    async def live(_):
        return web.json_response({"live": True})

    async def ready(_):
        ok = bool(getattr(backend, "ready", True))
        return web.json_response({"ready": ok}, status=200 if ok else 503)

    async def server_meta(_):
        return web.json_response({"name": "mlopamd-runtime", "version": "0.1.0",
                                  "extensions": ["generate", "metrics"]})

    async def model_meta(req):
        md = backend.metadata()
        md["versions"] = [version]
        return web.json_response(md)

    async def infer(req):
        body = await req.json()
        inputs = {i["name"]: i for i in body.get("inputs", [])}
        if backend.kind == "sklearn":
            first = next(iter(inputs.values()))
            x = np.asarray(first["data"], dtype=_DT.get(first.get("datatype", "FP32"), np.float32))
            x = x.reshape(first.get("shape", x.shape))
            y = backend.predict(x)
            y = np.asarray(y)
            dt = _DT_NAME.get(y.dtype, "BYTES")
            data = y.tolist() if dt != "BYTES" else [str(v) for v in y.tolist()]
            return web.json_response({"model_name": backend.name, "model_version": version,
                                      "id": body.get("id", ""), "outputs": [
                                          {"name": "predict", "shape": list(y.shape), "datatype": dt, "data": data}]})
        params = _params(body.get("parameters", {}))
        if "input_ids" in inputs:
            ids = [int(v) for v in inputs["input_ids"]["data"]]
            res = await backend.generate(ids, params)
            out = {"name": "output_ids", "shape": [len(res["output_ids"])], "datatype": "INT64",
                   "data": res["output_ids"]}
        else:
            text = inputs["text_input"]["data"][0]
            res = await backend.generate(backend.tokenizer.encode(text), params)
            out = {"name": "text_output", "shape": [1], "datatype": "BYTES",
                   "data": [backend.tokenizer.decode(res["output_ids"])]}
        return web.json_response({"model_name": backend.name, "model_version": version, "id": body.get("id", ""),
                                  "outputs": [out], "parameters": {"finish_reason": res["finish_reason"]}})

    async def generate(req):
        if backend.kind != "llm":
            raise web.HTTPBadRequest(text="generate is only served by LLM predictors")
        body = await req.json()
        params = _params(body.get("parameters", body))
        ids = body["input_ids"] if "input_ids" in body else backend.tokenizer.encode(body.get("text_input", ""))
        res = await backend.generate(ids, params)
        return web.json_response({"model_name": backend.name, "model_version": version,
                                  "text_output": backend.tokenizer.decode(res["output_ids"]),
                                  "output_ids": res["output_ids"], "finish_reason": res["finish_reason"],
                                  "usage": {"prompt_tokens": res["prompt_tokens"],
                                            "completion_tokens": len(res["output_ids"])},
                                  "ttft_s": res["ttft"], "latency_s": res["latency"]})

    async def generate_stream(req):
        if backend.kind != "llm":
            raise web.HTTPBadRequest(text="generate_stream is only served by LLM predictors")
        body = await req.json()
        params = _params(body.get("parameters", body))
        ids = body["input_ids"] if "input_ids" in body else backend.tokenizer.encode(body.get("text_input", ""))
        r = backend.submit(ids, params, stream=True)
        resp = web.StreamResponse(headers={"Content-Type": "text/event-stream"})
        await resp.prepare(req)
        while True:
            tok = await r.queue.get()
            if tok is None:
                break
            await resp.write(f"data: {json.dumps({'token_id': tok, 'text_output': backend.tokenizer.decode([tok])})}\n\n".encode())
        res = await r.future
        await resp.write(f"data: {json.dumps({'finish_reason': res['finish_reason'], 'done': True})}\n\n".encode())
        await resp.write_eof()
        return resp

    async def trace(_):
        eng = getattr(backend, "engine", None)
        if eng is None or not hasattr(eng, "tracer"):
            raise web.HTTPNotFound(text="no engine tracer on this predictor")
        return web.json_response(eng.tracer.chrome_trace())

    async def trace_summary(_):
        eng = getattr(backend, "engine", None)
        if eng is None or not hasattr(eng, "tracer"):
            raise web.HTTPNotFound(text="no engine tracer on this predictor")
        return web.json_response({"steps": eng.tracer.summary(), "stats": dict(eng.stats)})

    async def feedback(req):
        await req.read()
        return web.json_response({"status": "ok"})

    async def prom(_):
        if metrics is None:
            return web.Response(text="")
        try:
            from .gpu_metrics import sample

            metrics.update_gpu(sample())
        except Exception:  # noqa: BLE001
            pass
        return web.Response(body=metrics.exposition(), content_type="text/plain", charset="utf-8")

    r = app.router
    r.add_get("/v2/health/live", live)
    r.add_get("/v2/health/ready", ready)
    r.add_get("/v2", server_meta)
    r.add_get("/v2/models/{m}", model_meta)
    r.add_get("/v2/models/{m}/ready", ready)
    r.add_post("/v2/models/{m}/infer", infer)
    r.add_post("/v2/models/{m}/generate", generate)
    r.add_post("/v2/models/{m}/generate_stream", generate_stream)
    r.add_post("/api/v1.0/feedback", feedback)
    r.add_post("/api/v1.0/predictions", infer)
    r.add_get("/metrics", prom)
    r.add_get("/v2/debug/trace", trace)            # Chrome / Perfetto trace of recent engine steps
    r.add_get("/v2/debug/steps", trace_summary)

    async def startup(_):
        return web.json_response(STARTUP)

    async def on_start(_app):
        STARTUP["http_listening_s"] = _since_process_start()

    r.add_get("/v2/debug/startup", startup)
    app.on_startup.append(on_start)
    return app


def build_backend(runtime: str, model_uri: str | None, architecture: str | None, name: str, metrics,
                  device: str = "cuda", engine_kwargs: dict | None = None, seed: int = 0, tp_state=None):
    if runtime in ("mlop-sklearn", "sklearn"):
        from .backends import SklearnBackend

        return SklearnBackend(model_uri, name=name)
    from .backends import LLMBackend
    from .deploy import build_engine

    from .backends import load_tokenizer

    import torch

    t0 = time.perf_counter()
    STARTUP["engine_build_start_s"] = _since_process_start()
    dtype = {"float32": torch.float32, "bfloat16": torch.bfloat16}[os.environ.get("MLOP_DTYPE", "bfloat16")]
    eng = build_engine(architecture or "llama3-8b", device=device, seed=seed, tp_state=tp_state,
                       model_uri=model_uri, dtype=dtype, **(engine_kwargs or {}))
    STARTUP["engine_built_s"] = _since_process_start()
    STARTUP["engine"] = {k: int(eng.stats.get(k, 0)) for k in ("model_build_ms", "kv_alloc_ms", "graph_capture_ms")}
    from .. import ops

    # serving must never time GEMM candidates mid-request (a canary's latency would spike on
    # every first-seen batch size): decide from the shipped table / nearest tuned row count
    ops.freeze_autotune()
    if metrics is not None:
        metrics.load_seconds.labels(**metrics.labels).set(time.perf_counter() - t0)
        metrics.ready.labels(**metrics.labels).set(1)
    return LLMBackend(eng, metrics, tokenizer=load_tokenizer(eng.checkpoint_dir), name=name).start()


def engine_kwargs_from_env() -> dict:
    out = {}
    for k, v in os.environ.items():
        if k.startswith("MLOP_ENGINE_"):
            key = k[len("MLOP_ENGINE_"):].lower()
            try:
                out[key] = json.loads(v)
            except ValueError:
                out[key] = v
    return out


def main(argv=None):
    import sys

    argv = list(sys.argv[1:] if argv is None else argv)
    ap = argparse.ArgumentParser(description="mlopamd V2 inference server")
    ap.add_argument("--host", default="0.0.0.0")
    ap.add_argument("--port", type=int, default=int(os.environ.get("MLOP_PORT", 9000)))
    ap.add_argument("--runtime", default=os.environ.get("MLOP_RUNTIME", "mlop-llm"))
    ap.add_argument("--model-uri", default=os.environ.get("MLOP_MODEL_URI"))
    ap.add_argument("--architecture", default=os.environ.get("MLOP_ARCHITECTURE"))
    ap.add_argument("--name", default=os.environ.get("MLOP_MODEL_NAME", "model"))
    ap.add_argument("--version", default=os.environ.get("MLOP_MODEL_VERSION", "1"))
    ap.add_argument("--device", default=os.environ.get("MLOP_DEVICE", "cuda"))
    ap.add_argument("--tp", type=int, default=1)
    ap.add_argument("--ep", type=int, default=1,
                    help="expert-parallel degree with data-parallel attention (MoE; --tp 1): one "
                         "engine per GPU behind this endpoint (runtime/ep_serving.py)")
    ap.add_argument("--share-gpu", action="store_true",
                    help="one-GPU rehearsal of a --tp / --ep pod: every rank on device 0 over a gloo "
                         "group with the IPC all-reduce / exchange kernels forced (also MLOP_SHARE_GPU=1)")
    a = ap.parse_args(argv)
    if a.tp > 1 and a.ep > 1:
        raise SystemExit("--tp and --ep > 1 together: TP shards experts itself (EP = TP); use one")
    from .rank_launcher import launch_ranks, launcher_degree, share_gpu_requested

    a.share_gpu = share_gpu_requested(argv)
    n = launcher_degree(argv)
    if n > 1:  # main() called in-process (the __main__ path decided this before importing torch)
        raise SystemExit(launch_ranks(n, argv, a.share_gpu))

    from aiohttp import web

    from .metrics import RuntimeMetrics

    metrics = RuntimeMetrics(model_name=a.name)
    tp_state = None
    if a.ep > 1:
        from .ep_serving import serve_ep

        return serve_ep(a, metrics)
    if a.tp > 1 or int(os.environ.get("WORLD_SIZE", 1)) > 1:
        from .tp_worker import serve_tp

        return serve_tp(a, metrics)
    if os.environ.get("MLOP_INJECT_START_ERROR"):  # fault injection: e.g. a GPU OOM at weight load
        raise RuntimeError(os.environ["MLOP_INJECT_START_ERROR"])
    backend = build_backend(a.runtime, a.model_uri, a.architecture, a.name, metrics, a.device,
                            engine_kwargs_from_env(), tp_state=tp_state)
    crash_after = float(os.environ.get("MLOP_INJECT_CRASH_AFTER_S", 0) or 0)
    if crash_after > 0:  # fault injection: the process dies (SIGSEGV-like exit) after serving a while
        import threading

        threading.Timer(crash_after, lambda: os._exit(139)).start()
    web.run_app(make_app(backend, metrics, version=a.version), host=a.host, port=a.port, print=None)


if __name__ == "__main__":
    main()
