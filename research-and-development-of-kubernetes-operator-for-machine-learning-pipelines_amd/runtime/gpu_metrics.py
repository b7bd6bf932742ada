"""GPU telemetry for the per-pod exporter (G3): amd-smi, with a sysfs fallback.

``sample()`` returns one dict per GPU OF THIS POD: busy %, HBM used / total,
socket power.  The pod's GPUs are the devices the device plugin exported to it
(``HIP_VISIBLE_DEVICES`` / ``ROCR_VISIBLE_DEVICES``; every GPU when unset), so on
an 8-GPU node each predictor exports only its own cards and the canary's HBM /
power guards compare pods, not node totals.  Source order: the ``amdsmi``
Python bindings shipped with ROCm (/opt/rocm/share/amd_smi), then the amdgpu
sysfs files (gpu_busy_percent, mem_info_vram_used/total).  Everything is
best-effort: a box without either reports nothing rather than failing the
runtime.

``KernelTimeSampler`` profiles one engine step every ``period_s`` seconds in
process (torch.profiler over roctracer: the same kernel records rocprofv3
reads) and turns the kernels' device time into per-class shares (gemm /
attention / norm / rope_cache / moe / sampling / other) for the
``mlop_kernel_time_fraction`` gauge the canary gate can guard on;
``kernel_shares`` does the same for a rocprofv3 ``*_kernel_stats.csv``.
"""
from __future__ import annotations

import csv
import glob
import os
import sys

_amdsmi = None


def _init_amdsmi():
    global _amdsmi
    if _amdsmi is not None:
        return _amdsmi or None
    try:
        p = "/opt/rocm/share/amd_smi"
        if os.path.isdir(p) and p not in sys.path:
            sys.path.append(p)
        import amdsmi  # noqa: WPS433

        amdsmi.amdsmi_init()
        _amdsmi = amdsmi
    except Exception:  # noqa: BLE001
        _amdsmi = False
    return _amdsmi or None


def visible_devices() -> list[int] | None:
    """Physical indices of the GPUs this process (pod) was given, or None (all of them)."""
    for var in ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = os.environ.get(var)
        if v is not None and v.strip() != "":
            try:
                return [int(x) for x in v.split(",") if x.strip()]
            except ValueError:  # UUID-style lists: cannot map, report nothing rather than the node
                return []
    return None


def _sysfs() -> list[dict]:
    out = []
    cards = [d for d in sorted(glob.glob("/sys/class/drm/card*/device"))
             if os.path.exists(os.path.join(d, "gpu_busy_percent"))]
    for i, dev in enumerate(cards):
        def rd(name):
            try:
                with open(os.path.join(dev, name)) as f:
                    return float(f.read().strip())
            except (OSError, ValueError):
                return None
        busy = rd("gpu_busy_percent")
        if busy is None:
            continue
        out.append({"gpu": i, "busy_percent": busy, "mem_used": rd("mem_info_vram_used"),
                    "mem_total": rd("mem_info_vram_total"), "power_w": None, "source": "sysfs"})
    return out


def sample(devices: list[int] | None = ...) -> list[dict]:
    """One dict per GPU of this pod (``devices``: physical indices; default: the visible set)."""
    if devices is ...:
        devices = visible_devices()
    keep = (lambda i: True) if devices is None else (lambda i: i in devices)
    return [d for d in _sample_all() if keep(d["gpu"])]


def _sample_all() -> list[dict]:
    smi = _init_amdsmi()
    if smi is not None:
        out = []
        try:
            for i, h in enumerate(smi.amdsmi_get_processor_handles()):
                d = {"gpu": i, "source": "amdsmi"}
                try:
                    act = smi.amdsmi_get_gpu_activity(h)
                    d["busy_percent"] = float(act.get("gfx_activity", 0))
                except Exception:  # noqa: BLE001
                    d["busy_percent"] = None
                try:
                    d["mem_used"] = float(smi.amdsmi_get_gpu_memory_usage(h, smi.AmdSmiMemoryType.VRAM))
                    d["mem_total"] = float(smi.amdsmi_get_gpu_memory_total(h, smi.AmdSmiMemoryType.VRAM))
                except Exception:  # noqa: BLE001
                    d["mem_used"] = d["mem_total"] = None
                try:
                    pw = smi.amdsmi_get_power_info(h)
                    d["power_w"] = float(pw.get("current_socket_power") or pw.get("average_socket_power") or 0)
                except Exception:  # noqa: BLE001
                    d["power_w"] = None
                out.append(d)
            if out:
                return out
        except Exception:  # noqa: BLE001
            pass
    return _sysfs()


def classify_kernel(name: str) -> str:
    n = name.lower()
    if "moe_" in n:  # routing / sort / gather / combine (the expert GEMMs are gemm_* below)
        return "moe"
    if any(k in n for k in ("gemm", "gemv", "cijk", "mfma", "wsg_", "splitk_reduce")):
        return "gemm"
    if "attn" in n or "attention" in n or "flash" in n:
        return "attention"
    if "norm" in n:
        return "norm"
    if "rope" in n:
        return "rope_cache"
    if "sample" in n or "argmax" in n:
        return "sampling"
    return "other"


def kernel_shares(stats_csv: str) -> dict:
    """{class: fraction of total kernel time} from a rocprofv3 kernel_stats.csv."""
    tot, by = 0.0, {}
    with open(stats_csv) as f:
        for r in csv.DictReader(f):
            t = float(r["TotalDurationNs"])
            tot += t
            c = classify_kernel(r["Name"])
            by[c] = by.get(c, 0.0) + t
    return {k: v / tot for k, v in by.items()} if tot else {}


def shares_from_events(events) -> dict:
    """{class: fraction of device time} from (kernel name, device microseconds) pairs."""
    tot, by = 0.0, {}
    for name, us in events:
        if us <= 0:
            continue
        tot += us
        c = classify_kernel(name)
        by[c] = by.get(c, 0.0) + us
    return {k: v / tot for k, v in by.items()} if tot else {}


class KernelTimeSampler:
    """In-process kernel-time shares: every ``period_s`` the serving loop opens a ``torch.profiler``
    window (HIP activity) at one engine step and publishes the per-class device-time shares; the
    shares of a mixed / decode step are what a rocprof window of the pod would show (SURVEY.md
    §2.5 G3).

    Off the critical path: nothing ever waits for the device.  The profiled step gets an event
    after its launch; the window closes at the first later step boundary where that event has
    completed (``Event.query()``, non-blocking).  Under one-step-ahead scheduling that is the
    next step (the engine has read its tokens), so the window covers the profiled step plus at
    most the step queued behind it -- shares, not absolute times, are published.

    The engine thread only opens and stops the window; the event reduction (``key_averages``,
    the bulk of a window's host cost) runs on a helper thread (``MLOP_KERNEL_SAMPLE_ASYNC``,
    default on), and the first window opens one period after serving starts, never on the
    first step.  The tracer's one-time start-up (~2 s measured) is paid by ``warm`` on a
    background thread when the first window falls due; the window opens once it finished, so
    neither readiness, the first served requests nor a window's step waits for it
    (profiles/r06_sampler.md)."""

    def __init__(self, period_s: float | None = None, on_shares=None, async_reduce: bool | None = None):
        self.period_s = float(os.environ.get("MLOP_KERNEL_SAMPLE_S", 30.0) if period_s is None else period_s)
        self.on_shares = on_shares
        self.async_reduce = (os.environ.get("MLOP_KERNEL_SAMPLE_ASYNC", "1") not in ("0", "false", "")
                             if async_reduce is None else bool(async_reduce))
        self.last: dict = {}
        self._next = None  # first window: one period after the first step
        self._prof = None
        self._done_ev = None
        self.windows = 0
        # the sampler's own cost ON THE ENGINE THREAD (opening + closing [+ reducing] a window),
        # per window, and the one-time tracer start-up paid in ``warm``
        self.host_ms: list = []
        self.reduce_ms: list = []
        self._open_ms = 0.0
        self.warm_ms = None
        self._warm_thread = None
        self._reducer = None

    def warm(self, background: bool = False) -> None:
        """Pay the tracer's one-time start-up (profiler library + HIP activity callbacks) with a
        throwaway window around one tiny kernel, instead of inside the first served window,
        where it stalled the step loop.  ``background``: on a daemon thread (the predictor's
        readiness does not wait for it; a window opens only after it finished)."""
        import time

        if self.period_s <= 0 or self.warm_ms is not None or self._warm_thread is not None:
            return
        import torch

        if not torch.cuda.is_available():
            return

        def run():
            t0 = time.perf_counter()
            dev = torch.cuda.current_device()
            with torch.profiler.profile(activities=[torch.profiler.ProfilerActivity.CUDA]) as p:
                with torch.cuda.device(dev):
                    torch.ones(1, device="cuda").add_(1)
                    torch.cuda.synchronize()
            p.key_averages()
            self.warm_ms = round(1e3 * (time.perf_counter() - t0), 3)

        if background:
            import threading

            dev = torch.cuda.current_device()

            def bg():
                torch.cuda.set_device(dev)
                run()

            self._warm_thread = threading.Thread(target=bg, name="ktime-warm", daemon=True)
            self._warm_thread.start()
        else:
            run()

    def before_step(self, now: float) -> None:
        if self.period_s <= 0 or self._prof is not None:
            return
        if self._next is None:
            self._next = now + self.period_s
            return
        if now < self._next:
            return
        if self.warm_ms is None:
            # first due window: start the tracer's one-time start-up on its own thread now (not at
            # predictor start, where its ~2 s of GIL-holding work slowed the first served requests
            # -- a fresh canary's -- ~10x: profiles/r06_sampler.md), open the window once it is done
            if self._warm_thread is None:
                self.warm(background=True)
            if self._warm_thread is not None and self._warm_thread.is_alive():
                return
        if self._warm_thread is not None and self._warm_thread.is_alive():
            return  # the tracer is still starting on its own thread
        if self._reducer is not None and self._reducer.is_alive():
            return  # the previous window is still being reduced
        import time

        import torch

        if not torch.cuda.is_available():
            return
        t0 = time.perf_counter()
        self._prof = torch.profiler.profile(activities=[torch.profiler.ProfilerActivity.CUDA])
        self._prof.__enter__()
        self._open_ms = 1e3 * (time.perf_counter() - t0)

    def after_step(self, now: float) -> dict | None:
        if self._prof is None:
            return None
        import time

        import torch

        if self._done_ev is None:  # the profiled step was just launched: mark its end
            self._done_ev = torch.cuda.Event()
            self._done_ev.record()
            return None
        if not self._done_ev.query():  # still running: look again after the next step
            return None
        t0 = time.perf_counter()
        prof = self._prof
        prof.__exit__(None, None, None)
        self._prof, self._done_ev = None, None
        self._next = now + self.period_s
        self.windows += 1
        if self.async_reduce:
            import threading

            self.host_ms.append(round(self._open_ms + 1e3 * (time.perf_counter() - t0), 3))
            del self.host_ms[:-64]
            self._reducer = threading.Thread(target=self._reduce, args=(prof,), name="ktime-reduce", daemon=True)
            self._reducer.start()
            return None
        shares = self._reduce(prof)
        self.host_ms.append(round(self._open_ms + 1e3 * (time.perf_counter() - t0), 3))
        del self.host_ms[:-64]
        return shares

    def _reduce(self, prof) -> dict:
        import time

        t0 = time.perf_counter()
        ev = [(e.key, float(getattr(e, "device_time_total", 0.0) or getattr(e, "cuda_time_total", 0.0)))
              for e in prof.key_averages()]
        shares = shares_from_events(ev)
        self.reduce_ms.append(round(1e3 * (time.perf_counter() - t0), 3))
        del self.reduce_ms[:-64]
        if shares:
            self.last = shares
            if self.on_shares is not None:
                self.on_shares(shares)
        return shares

    def join(self, timeout: float = 30.0) -> None:
        """Wait for a pending background warm-up / reduction (tests, benches)."""
        for t in (self._warm_thread, self._reducer):
            if t is not None:
                t.join(timeout)
