"""Engine tracing (SURVEY.md §5 "tracing / profiling"; the reference has none).

* ``StepTracer`` — an always-on ring buffer of engine-step spans (kind, decode /
  prefill token counts, host-prep / device / bookkeeping time) that costs two
  ``perf_counter`` calls per step; exported as a Chrome / Perfetto trace
  (``/v2/debug/trace`` on the runtime server) so a serving timeline can be
  read next to a ``rocprofv3 --kernel-trace`` of the same run.
* ``TorchProfileWindow`` — ``MLOP_PROFILE_STEPS=a:b`` wraps engine steps a..b in
  ``torch.profiler`` (CPU + HIP activities) and writes a Chrome trace to
  ``MLOP_PROFILE_DIR`` (default ``gpurun_out/torch_profile``).
"""
from __future__ import annotations

import collections
import json
import os
import time


class StepTracer:
    def __init__(self, capacity: int = 4096):
        self.spans: collections.deque = collections.deque(maxlen=capacity)
        self.t0 = time.perf_counter()
        self.n = 0

    def record(self, kind: str, t_start: float, t_end: float, **args):
        self.n += 1
        self.spans.append((kind, t_start, t_end, args))

    def summary(self) -> dict:
        by = collections.defaultdict(lambda: [0, 0.0])
        for kind, a, b, _ in self.spans:
            by[kind][0] += 1
            by[kind][1] += b - a
        return {k: {"steps": n, "mean_ms": round(1e3 * t / max(n, 1), 3)} for k, (n, t) in by.items()}

    def chrome_trace(self) -> dict:
        ev = []
        for i, (kind, a, b, args) in enumerate(self.spans):
            ev.append({"name": kind, "ph": "X", "pid": os.getpid(), "tid": 0,
                       "ts": round(1e6 * (a - self.t0), 1), "dur": round(1e6 * (b - a), 1),
                       "args": dict(args, step=self.n - len(self.spans) + i)})
        return {"traceEvents": ev, "displayTimeUnit": "ms"}

    def dump(self, path: str):
        with open(path, "w") as f:
            json.dump(self.chrome_trace(), f)


class TorchProfileWindow:
    """Profile engine steps [start, stop) with torch.profiler when MLOP_PROFILE_STEPS is set."""

    def __init__(self, spec: str | None = None, out_dir: str | None = None):
        spec = spec if spec is not None else os.environ.get("MLOP_PROFILE_STEPS", "")
        self.start = self.stop = -1
        if spec:
            a, b = spec.split(":")
            self.start, self.stop = int(a), int(b)
        self.out_dir = out_dir or os.environ.get("MLOP_PROFILE_DIR", "gpurun_out/torch_profile")
        self.prof = None
        self.step_i = 0

    @property
    def enabled(self) -> bool:
        return self.start >= 0

    def before_step(self):
        if self.enabled and self.step_i == self.start and self.prof is None:
            import torch

            acts = [torch.profiler.ProfilerActivity.CPU]
            if torch.cuda.is_available():
                acts.append(torch.profiler.ProfilerActivity.CUDA)
            self.prof = torch.profiler.profile(activities=acts, record_shapes=False)
            self.prof.__enter__()

    def after_step(self):
        self.step_i += 1
        if self.prof is not None and self.step_i >= self.stop:
            self.prof.__exit__(None, None, None)
            os.makedirs(self.out_dir, exist_ok=True)
            path = os.path.join(self.out_dir, f"engine_steps_{self.start}_{self.stop}_{os.getpid()}.json")
            self.prof.export_chrome_trace(path)
            self.prof = None
            self.start = -1  # one window per process
