"""GPU telemetry for the per-pod exporter (G3): amd-smi, with a sysfs fallback.

``sample()`` returns one dict per visible GPU: busy %, HBM used / total,
socket power.  Source order: the ``amdsmi`` Python bindings shipped with ROCm
(/opt/rocm/share/amd_smi), then the amdgpu sysfs files
(gpu_busy_percent, mem_info_vram_used/total).  Everything is best-effort: a
box without either reports nothing rather than failing the runtime.

``KernelTimeSampler`` turns a rocprofv3 ``*_kernel_stats.csv`` into per-class
time shares (gemm / attention / norm / other) for the same exporter.
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


def _sysfs() -> list[dict]:
    out = []
    for i, dev in enumerate(sorted(glob.glob("/sys/class/drm/card*/device"))):
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


def sample() -> list[dict]:
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
    if "gemm" in n or "cijk" in n or "mfma" in n:
        return "gemm"
    if "attn" in n or "attention" in n:
        return "attention"
    if "norm" in n:
        return "norm"
    if "rope" in n:
        return "rope_cache"
    if "sample" in n or "argmax" in n:
        return "sampling"
    if "moe" in n:
        return "moe"
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
