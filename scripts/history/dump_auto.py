"""Run bench.py in-process with MLOP_GEMM_BACKEND=auto and dump the per-shape timings the
backend every (M bucket, N, K, epilogue) key ran on (gpurun_out/auto_times.json): which (M bucket, N, K, epilogue) keys went
to hipBLASLt and by how much."""
import atexit
import json
import os
import runpy
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
os.environ["MLOP_GEMM_BACKEND"] = "auto"
from mlopamd import ops  # noqa: E402


def dump():
    # the shipped table seeds the choices and bench.py freezes them, so report what RAN
    rows = [{"key": list(k), "backend": v, "table_times_us": ops._GEMM_TIMES.get(k)} for k, v in ops._GEMM_USED.items()]
    rows.sort(key=lambda r: (r["key"][0], r["key"][1]))
    os.makedirs("gpurun_out", exist_ok=True)
    with open("gpurun_out/auto_times.json", "w") as f:
        json.dump(rows, f, indent=1)


atexit.register(dump)
sys.argv = ["bench.py"] + sys.argv[1:]
runpy.run_path(os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "bench.py"),
               run_name="__main__")
