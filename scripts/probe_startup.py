"""Predictor start-up probe: how long do `import torch` and the first device allocation take in a
fresh process, and does initialising the HIP runtime on a helper thread WHILE torch imports
(ctypes hipInit / hipSetDevice / hipFree(0): the GIL is released inside the C calls) take the
device initialisation off the critical path?  Each variant runs in 3 fresh child processes.

    python3 scripts/probe_startup.py
"""
import json
import subprocess
import sys

CHILD = r'''
import time, threading, ctypes, os, json
t0 = time.perf_counter()
mode = os.environ["PROBE_MODE"]
th = None
if mode == "thread":
    def warm():
        import importlib.util
        spec = importlib.util.find_spec("torch")
        lib = ctypes.CDLL(os.path.join(os.path.dirname(spec.origin), "lib", "libamdhip64.so"))
        lib.hipInit(0)
        lib.hipSetDevice(0)
        lib.hipFree(ctypes.c_void_p(0))
    th = threading.Thread(target=warm)
    th.start()
import torch
t1 = time.perf_counter()
if th is not None:
    th.join()
t2 = time.perf_counter()
x = torch.zeros(1, device="cuda")
torch.cuda.synchronize()
t3 = time.perf_counter()
hip = sorted({l.split()[-1] for l in open("/proc/self/maps") if "amdhip" in l})
print(json.dumps({"mode": mode, "hip_runtimes": hip, "import_torch_s": round(t1 - t0, 3), "join_s": round(t2 - t1, 3),
                  "first_alloc_s": round(t3 - t2, 3), "total_s": round(t3 - t0, 3)}), flush=True)
'''


def main():
    for mode in ("plain", "thread", "plain", "thread", "plain", "thread"):
        env = dict(__import__("os").environ, PROBE_MODE=mode)
        out = subprocess.run([sys.executable, "-c", CHILD], env=env, capture_output=True, text=True, timeout=300)
        line = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
        print(line[-1] if line else json.dumps({"mode": mode, "error": out.stderr[-400:]}), flush=True)


if __name__ == "__main__":
    main()
