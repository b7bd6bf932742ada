"""In-tree build of the gfx950 HIP extension (``ops/_C.so``).

Every ``csrc/*.hip`` file is compiled by ``hipcc --offload-arch=gfx950`` into
its own object (parallel, incremental on CONTENT: an object is rebuilt when the
hash of its source + every header + its command line differs from the one
recorded beside it, never on mtimes), ``csrc/bindings.cpp`` (the torch op
registrations) is compiled against torch's headers, and the objects are linked
against torch's own HIP runtime (``torch/lib/libamdhip64.so``, SONAME
``libamdhip64.so.7``) so the process holds exactly one HIP runtime.

Build integrity: the sha256 of all sources (``source_hash()``) is compiled INTO the
library (``torch.ops.mlop.src_hash()``); ``ops.load()`` refuses a ``_C.so`` whose
embedded hash differs from the tree it is loaded from (a stale or foreign binary).

No hipify, no cpp_extension JIT cache: the ``.so`` lives next to this file and
travels with the repo snapshot to the GPU box.

Usage: ``python -m mlopamd.ops.build [-j N] [--force]``.
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import hashlib
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


def _sources() -> list[Path]:
    return sorted([*CSRC.glob("*.hip"), *CSRC.glob("*.h"), *CSRC.glob("*.cpp"), *CSRC.glob("*.cc")])


def source_hash() -> str:
    """sha256 over every HIP / C++ source and header, the per-file flags and the target arch."""
    h = hashlib.sha256()
    for f in _sources():
        h.update(f.name.encode() + b"\0" + f.read_bytes() + b"\0")
    h.update(repr(sorted(FILE_FLAGS.items())).encode() + ARCH.encode())
    return h.hexdigest()[:32]


def _stale(obj: Path, src: Path, headers, cmd) -> tuple[bool, str]:
    h = hashlib.sha256(src.read_bytes())
    for d in headers:
        h.update(d.read_bytes())
    h.update(" ".join(map(str, cmd)).encode())
    digest = h.hexdigest()
    side = obj.with_suffix(".sha")
    return (not obj.exists() or not side.exists() or side.read_text() != digest), digest


# Per-file code-generation flags.  attention: no NaN operands assumed (the masks use -inf,
# which stays honoured), so fmaxf on MFMA results needs no canonicalising v_max first: -16 of
# the flash-prefill loop's ~215 VALU instructions per 32-key step (the loop is VALU-issue
# bound, profiles/r02_flash_prefill.md).  NaN scores give unspecified (not NaN-propagating)
# attention outputs.  -fno-slp-vectorize: no v_pk_mul_f32 / v_pk_add_f32 from adjacent f32 ops
# (the O rescale): a packed f32 op beside MFMAs costs ~22-26 cycles more than two scalar ones
# (MI355X_MICROARCH.md, per-instruction constants).
FILE_FLAGS = {"attention": ["-fno-honor-nans", "-fno-slp-vectorize"]}


def _run(cmd):
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError("build failed:\n" + " ".join(map(str, cmd)) + "\n" + r.stdout + r.stderr)
    return r


def build(jobs: int | None = None, force: bool = False, verbose: bool = False) -> Path:
    hipcc = _hipcc()
    troot, tinc, abi = _torch_dirs()
    BUILD.mkdir(exist_ok=True)
    headers = sorted(CSRC.glob("*.h"))
    kernels = sorted(CSRC.glob("*.hip"))
    # -Werror=return-type: a value-returning function that falls off its end is UB (a host crash)
    common = ["-O3", "-std=c++17", "-fPIC", f"-I{CSRC}", "-D__HIP_PLATFORM_AMD__=1", "-Werror=return-type"]
    jobs_list = []  # (cmd, obj, digest)
    for src in kernels:
        obj = BUILD / (src.stem + ".o")
        cmd = [hipcc, *common, f"--offload-arch={ARCH}", "-ffp-contract=fast",
               *FILE_FLAGS.get(src.stem, []), "-c", str(src), "-o", str(obj)]
        stale, digest = _stale(obj, src, headers, cmd)
        if force or stale:
            jobs_list.append((cmd, obj, digest))
    # host-only runtime sources (C++, no device code): csrc/*.cc
    hosts = sorted(CSRC.glob("*.cc"))
    for src in hosts:
        obj = BUILD / (src.stem + ".o")
        cmd = [hipcc, *common, "-x", "c++", "-c", str(src), "-o", str(obj)]
        stale, digest = _stale(obj, src, headers, cmd)
        if force or stale:
            jobs_list.append((cmd, obj, digest))
    bsrc = CSRC / "bindings.cpp"
    bobj = BUILD / "bindings.o"
    py_inc = sysconfig.get_paths()["include"]
    bcmd = [hipcc, *common, "-x", "c++", f"-D_GLIBCXX_USE_CXX11_ABI={abi}", "-DUSE_ROCM=1",
            "-DTORCH_EXTENSION_NAME=_C", *[f"-I{p}" for p in tinc], f"-I{py_inc}",
            "-I/opt/rocm/include", "-Wno-deprecated-declarations",
            "-c", str(bsrc), "-o", str(bobj)]
    stale, digest = _stale(bobj, bsrc, headers, bcmd)
    if force or stale:
        jobs_list.append((bcmd, bobj, digest))
    # the tree's source hash, compiled into the library (ops.load() checks it)
    want = source_hash()
    hsrc, hobj = BUILD / "srchash.cpp", BUILD / "srchash.o"
    body = f'extern "C" const char* mlop_src_hash() {{ return "{want}"; }}\n'
    if force or not hsrc.exists() or hsrc.read_text() != body or not hobj.exists():
        hsrc.write_text(body)
        jobs_list.append(([hipcc, "-O2", "-fPIC", "-x", "c++", "-c", str(hsrc), "-o", str(hobj)], hobj, None))
    n = jobs or min(len(jobs_list), max(1, (os.cpu_count() or 4) // 2), 16) or 1

    def run(job):
        cmd, obj, digest = job
        r = _run(cmd)
        if digest is not None:
            obj.with_suffix(".sha").write_text(digest)
        return r

    if jobs_list:
        with cf.ThreadPoolExecutor(max_workers=n) as ex:
            for r in ex.map(run, jobs_list):
                if verbose and (r.stdout or r.stderr):
                    print(r.stdout, r.stderr, file=sys.stderr)
    objs = [BUILD / (s.stem + ".o") for s in kernels] + [BUILD / (s.stem + ".o") for s in hosts] + [bobj, hobj]
    if force or jobs_list or not OUT.exists():
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
