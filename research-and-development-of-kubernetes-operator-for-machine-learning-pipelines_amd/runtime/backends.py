"""Model backends hosted by the runtime server.

* ``LLMBackend`` — owns an ``Engine`` on a dedicated thread (the GPU is driven
  from exactly one host thread); HTTP handlers submit requests through a
  lock-protected queue and await futures resolved from the engine thread
  (``loop.call_soon_threadsafe``).  Streaming yields tokens as they come.
* ``SklearnBackend`` — CPU tabular models for BASELINE config 1 (sklearn-iris):
  a safe JSON linear-model format written by ``save_linear_model`` (no
  pickle), and MLflow ``sklearn`` flavour pickles only when
  ``MLOP_ALLOW_PICKLE=1`` (trusted, self-written artifacts).
* ``ByteTokenizer`` — reversible UTF-8 byte tokenizer (ids 3..258), so text
  I/O works offline with random-init weights.
"""
from __future__ import annotations

import asyncio
import json
import os
import threading
import time
from pathlib import Path

import numpy as np

from .sampler import SamplingParams


class ByteTokenizer:
    offset = 3
    eos_id = 1

    def encode(self, text: str) -> list[int]:
        return [b + self.offset for b in text.encode("utf-8")] or [self.offset]

    def decode(self, ids) -> str:
        return bytes(max(0, min(255, i - self.offset)) for i in ids if i >= self.offset).decode("utf-8", "replace")


class HFTokenizer:
    """A checkpoint's ``tokenizer.json`` (Hugging Face ``tokenizers``, no network)."""

    def __init__(self, path):
        from tokenizers import Tokenizer

        self._tok = Tokenizer.from_file(str(path))

    def encode(self, text: str) -> list[int]:
        return self._tok.encode(text).ids

    def decode(self, ids) -> str:
        return self._tok.decode(list(ids), skip_special_tokens=True)


def load_tokenizer(checkpoint_dir):
    """The checkpoint's own tokenizer when it ships one, else the byte tokenizer."""
    if checkpoint_dir is not None:
        p = Path(checkpoint_dir) / "tokenizer.json"
        if p.is_file():
            return HFTokenizer(p)
    return ByteTokenizer()


class _Req:
    __slots__ = ("prompt", "params", "loop", "future", "queue", "tokens", "t0", "t_first", "seq")

    def __init__(self, prompt, params, loop, stream):
        self.prompt, self.params, self.loop = prompt, params, loop
        self.future = loop.create_future()
        self.queue = asyncio.Queue() if stream else None
        self.tokens, self.t0, self.t_first, self.seq = [], time.perf_counter(), None, None


class LLMBackend:
    kind = "llm"

    def __init__(self, engine, metrics=None, tokenizer=None, name: str = "model"):
        self.engine, self.metrics, self.name = engine, metrics, name
        self.tokenizer = tokenizer or ByteTokenizer()
        self._pending: list[_Req] = []
        self._active: dict[int, _Req] = {}
        self._lock = threading.Lock()
        self._wake = threading.Event()
        self._stop = False
        self._thread = threading.Thread(target=self._loop, name="mlop-engine", daemon=True)
        self.steps = 0
        from .gpu_metrics import KernelTimeSampler

        # one profiled engine step per period -> mlop_kernel_time_fraction{kernel=...}
        self.ktime = KernelTimeSampler(on_shares=metrics.update_kernel_shares if metrics is not None else None)

    @property
    def ready(self) -> bool:
        return self._thread.is_alive()

    def start(self):
        self._thread.start()
        return self

    def stop(self):
        self._stop = True
        self._wake.set()
        self._thread.join(timeout=10)

    # ----- engine thread -----
    def _loop(self):
        eng = self.engine
        while not self._stop:
            with self._lock:
                pend, self._pending = self._pending, []
            for r in pend:
                try:
                    r.seq = eng.add_request(r.prompt, r.params)
                    self._active[r.seq.seq_id] = r
                except Exception as e:  # noqa: BLE001
                    r.loop.call_soon_threadsafe(_set_exc, r.future, e)
            if not eng.has_work():
                self._wake.wait(0.05)
                self._wake.clear()
                continue
            self.ktime.before_step(time.perf_counter())
            outs = eng.step()
            self.steps += 1
            now = time.perf_counter()
            self.ktime.after_step(now)
            if self.metrics:
                self.metrics.mark_step(len(outs), now)
            for o in outs:
                r = self._active.get(o.seq_id)
                if r is None:
                    continue
                if r.t_first is None:
                    r.t_first = now
                    if self.metrics:
                        self.metrics.ttft.labels(**self.metrics.labels).observe(now - r.t0)
                        self.metrics.tokens_in.labels(**self.metrics.labels).inc(len(r.prompt))
                r.tokens.append(o.token)
                if r.queue is not None:
                    r.loop.call_soon_threadsafe(r.queue.put_nowait, o.token)
                if o.finished:
                    self._active.pop(o.seq_id, None)
                    res = {"output_ids": list(r.tokens), "finish_reason": o.finish_reason,
                           "ttft": r.t_first - r.t0, "latency": now - r.t0,
                           "prompt_tokens": len(r.prompt)}
                    if self.metrics:
                        m = self.metrics
                        m.tokens_out.labels(**m.labels).inc(len(r.tokens))
                        if len(r.tokens) > 1:
                            m.tpot.labels(**m.labels).observe((now - r.t_first) / (len(r.tokens) - 1))
                    if r.queue is not None:
                        r.loop.call_soon_threadsafe(r.queue.put_nowait, None)
                    r.loop.call_soon_threadsafe(_set_res, r.future, res)
            if self.metrics:
                m = self.metrics
                m.running.labels(**m.labels).set(eng.num_running)
                m.waiting.labels(**m.labels).set(len(eng.waiting))
                m.kv_usage.labels(**m.labels).set(eng.kv_usage())
                m.kv_blocks.labels(**m.labels).set(eng.alloc.available)
                m.kv_fill_failed.labels(**m.labels).set(1 if eng.stats.get("kv_fill_failed") else 0)

    # ----- asyncio side -----
    def submit(self, prompt_ids, params: SamplingParams, stream: bool = False) -> _Req:
        r = _Req(list(prompt_ids), params, asyncio.get_running_loop(), stream)
        with self._lock:
            self._pending.append(r)
        self._wake.set()
        return r

    async def generate(self, prompt_ids, params: SamplingParams) -> dict:
        return await self.submit(prompt_ids, params).future

    def metadata(self) -> dict:
        cfg = self.engine.model.cfg
        return {"name": self.name, "platform": "mlopamd-llm-rocm", "architecture": cfg.name,
                "inputs": [{"name": "text_input", "datatype": "BYTES", "shape": [-1]},
                           {"name": "input_ids", "datatype": "INT64", "shape": [-1]}],
                "outputs": [{"name": "text_output", "datatype": "BYTES", "shape": [-1]},
                            {"name": "output_ids", "datatype": "INT64", "shape": [-1]}]}


def _set_res(fut, res):
    if not fut.done():
        fut.set_result(res)


def _set_exc(fut, e):
    if not fut.done():
        fut.set_exception(e)


# ----------------------------------------------------------------- sklearn --

def save_linear_model(path: str | Path, coef, intercept, classes, kind: str = "logistic_regression",
                      feature_names=None) -> Path:
    """Write a model dir: MLmodel (flavour 'mlop_linear') + model.json (no pickle)."""
    p = Path(path)
    p.mkdir(parents=True, exist_ok=True)
    (p / "model.json").write_text(json.dumps({
        "type": kind, "coef": np.asarray(coef).tolist(), "intercept": np.asarray(intercept).tolist(),
        "classes": np.asarray(classes).tolist(), "feature_names": feature_names}))
    (p / "MLmodel").write_text("flavors:\n  mlop_linear:\n    data: model.json\n  python_function:\n"
                               "    loader_module: mlopamd.runtime.backends\n")
    return p


def local_path(uri: str) -> Path:
    if uri.startswith("file://"):
        return Path(uri[len("file://"):])
    if "://" in uri:
        # s3://mlflow/<rel> -> MLOP_ARTIFACT_ROOT/<rel> (the storage initializer's job in Seldon)
        root = os.environ.get("MLOP_ARTIFACT_ROOT", "/mnt/models")
        return Path(root) / uri.split("://", 1)[1].split("/", 1)[-1]
    return Path(uri)


class SklearnBackend:
    kind = "sklearn"

    def __init__(self, model_uri: str, name: str = "model"):
        self.name = name
        p = local_path(model_uri)
        if (p / "model.json").exists():
            m = json.loads((p / "model.json").read_text())
            self.coef = np.asarray(m["coef"], dtype=np.float64)
            self.intercept = np.asarray(m["intercept"], dtype=np.float64)
            self.classes = np.asarray(m["classes"])
            self.type = m["type"]
            self._sk = None
        elif (p / "model.pkl").exists() and os.environ.get("MLOP_ALLOW_PICKLE") == "1":
            import pickle  # noqa: S403 - trusted, self-written artifacts only (opt-in)

            with open(p / "model.pkl", "rb") as f:
                self._sk = pickle.load(f)  # noqa: S301
            self.type = "sklearn"
        else:
            raise FileNotFoundError(f"no loadable model at {p} (model.json, or model.pkl with MLOP_ALLOW_PICKLE=1)")
        self.ready = True

    def predict(self, x: np.ndarray) -> np.ndarray:
        x = np.asarray(x, dtype=np.float64)
        if self._sk is not None:
            return np.asarray(self._sk.predict(x))
        z = x @ self.coef.T + self.intercept
        if self.type == "linear_regression":
            return z.ravel() if z.ndim == 2 and z.shape[1] == 1 else z
        if z.ndim == 1 or z.shape[1] == 1:
            return self.classes[(z.ravel() > 0).astype(int)]
        return self.classes[np.argmax(z, axis=1)]

    def metadata(self) -> dict:
        return {"name": self.name, "platform": "mlopamd-sklearn", "inputs": [
            {"name": "input-0", "datatype": "FP32", "shape": [-1, int(self.coef.shape[-1]) if self._sk is None else -1]}],
            "outputs": [{"name": "predict", "datatype": "INT64", "shape": [-1]}]}
