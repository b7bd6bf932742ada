"""In-tree build of the gfx950 HIP extension (``ops/_C.so``).

Every ``csrc/*.hip`` file is compiled by ``hipcc --offload-arch=gfx950`` into
its own object (parallel, incremental on mtimes), ``csrc/bindings.cpp`` (the
torch op registrations) is compiled against torch's headers, and the objects
are linked against torch's own HIP runtime (``torch/lib/libamdhip64.so``,
SONAME ``libamdhip64.so.7``) so the process holds exactly one HIP runtime.

No hipify, no cpp_extension JIT cache: the ``.so`` lives next to this file and
travels with the repo snapshot to the GPU box.

Usage: ``python -m mlopamd.ops.build [-j N] [--force]``.
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import os
import shutil
import subprocess
import sys
import sysconfig
from pathlib import Path

HERE = Path(__file__).resolve().parent
CSRC = HERE / "csrc"
BUILD = HERE / "_build"
OUT = HERE / "_C.so"
ARCH = os.environ.get("MLOP_OFFLOAD_ARCH", "gfx950")


def _hipcc() -> str:
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found (ROCm toolchain required to build the extension)")


def _torch_dirs():
    import torch  # noqa: WPS433 (build-time only)

    root = Path(torch.__file__).resolve().parent
    inc = [root / "include", root / "include" / "torch" / "csrc" / "api" / "include"]
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    return root, inc, abi


def _newer(target: Path, deps) -> bool:
    if not target.exists():
        return True
    t = target.stat().st_mtime
    return any(d.stat().st_mtime > t for d in deps)


# Per-file code-generation flags.  attention: no NaN operands assumed (the masks use -inf,
# which stays honoured), so fmaxf on MFMA results needs no canonicalising v_max first: -16 of
# the flash-prefill loop's ~215 VALU instructions per 32-key step (the loop is VALU-issue
# bound, profiles/r02_flash_prefill.md).  NaN scores give unspecified (not NaN-propagating)
# attention outputs.
FILE_FLAGS = {"attention": ["-fno-honor-nans"]}


def _run(cmd):
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError("build failed:\n" + " ".join(map(str, cmd)) + "\n" + r.stdout + r.stderr)
    return r


def build(jobs: int | None = None, force: bool = False, verbose: bool = False) -> Path:
    hipcc = _hipcc()
    troot, tinc, abi = _torch_dirs()
    BUILD.mkdir(exist_ok=True)
    headers = list(CSRC.glob("*.h"))
    kernels = sorted(CSRC.glob("*.hip"))
    common = ["-O3", "-std=c++17", "-fPIC", f"-I{CSRC}", "-D__HIP_PLATFORM_AMD__=1"]
    jobs_list = []
    for src in kernels:
        obj = BUILD / (src.stem + ".o")
        if force or _newer(obj, [src, *headers, Path(__file__)]):
            cmd = [hipcc, *common, f"--offload-arch={ARCH}", "-ffp-contract=fast",
                   *FILE_FLAGS.get(src.stem, []), "-c", str(src), "-o", str(obj)]
            jobs_list.append(cmd)
    bsrc = CSRC / "bindings.cpp"
    bobj = BUILD / "bindings.o"
    if force or _newer(bobj, [bsrc, *headers]):
        py_inc = sysconfig.get_paths()["include"]
        cmd = [hipcc, *common, "-x", "c++", f"-D_GLIBCXX_USE_CXX11_ABI={abi}", "-DUSE_ROCM=1",
               "-DTORCH_EXTENSION_NAME=_C", *[f"-I{p}" for p in tinc], f"-I{py_inc}",
               "-I/opt/rocm/include", "-Wno-deprecated-declarations",
               "-c", str(bsrc), "-o", str(bobj)]
        jobs_list.append(cmd)
    n = jobs or min(len(jobs_list), max(1, (os.cpu_count() or 4) // 2), 16) or 1
    if jobs_list:
        with cf.ThreadPoolExecutor(max_workers=n) as ex:
            for r in ex.map(_run, jobs_list):
                if verbose and (r.stdout or r.stderr):
                    print(r.stdout, r.stderr, file=sys.stderr)
    objs = [BUILD / (s.stem + ".o") for s in kernels] + [bobj]
    if force or jobs_list or _newer(OUT, objs):
        tlib = troot / "lib"
        tmp = OUT.with_suffix(".so.tmp")
        cmd = [hipcc, "-shared", "-fPIC", f"--offload-arch={ARCH}", *map(str, objs),
               f"-L{tlib}", "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu", "-ltorch_hip",
               "-lamdhip64", f"-Wl,-rpath,{tlib}", "-o", str(tmp)]
        _run(cmd)
        os.replace(tmp, OUT)
    return OUT


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("-j", "--jobs", type=int, default=None)
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-v", "--verbose", action="store_true")
    a = ap.parse_args(argv)
    print(build(a.jobs, a.force, a.verbose))


if __name__ == "__main__":
    main()
