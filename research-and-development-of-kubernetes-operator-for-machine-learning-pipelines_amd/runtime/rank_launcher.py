"""The multi-rank predictor pod's launcher (configs 4 and 5 as the operator ships them).

The SeldonDeployment's predictor command is plain ``python -m mlopamd.runtime.server --tp N``
(or ``--ep N``) with no rank launcher around it (controller/seldon.py).  That process becomes
the launcher of N rank processes and stays a pure process supervisor:

  * it decides its role from argv and env ALONE, before ``import torch`` and before any HIP
    call (``launcher_degree``): no device context, no ``/dev/kfd`` descriptor, no HIP warm-up
    thread in the launcher — only the ranks touch the GPU, and a launcher that initialised
    HIP before forking would hold a context on the pod's first GPU for its whole life;
  * rank r gets ``LOCAL_RANK=r`` (an index into the pod's ``HIP_VISIBLE_DEVICES``), the
    rendezvous on 127.0.0.1 and ``HSA_ENABLE_IPC_MODE_LEGACY=0`` (dmabuf IPC: K15 / the EP
    exchange map peer buffers);
  * ``--share-gpu`` (or ``MLOP_SHARE_GPU=1`` in the pod env) is the one-GPU rehearsal: every
    rank on device 0 over a gloo process group with the K15 IPC kernels forced (RCCL refuses
    two ranks on one device), exactly like ``bench.py --share-gpu``;
  * the first rank to exit ends the group (the rest are terminated, rank 0 first so its
    shutdown releases the parked workers) and the launcher exits with that status: the kubelet
    (or the local Seldon stand-in) sees one pod that failed, as with ``torchrun``.

Reference contract: one predictor per model version (``/root/reference/mlflow_operator.py:194-222``)
— with TP / EP it is one pod of N ranks.
"""
from __future__ import annotations

import json
import os
import signal
import socket
import subprocess
import sys
import time

# what the launcher reports to its ranks (rank 0 serves it at /v2/debug/startup): proof that
# the launcher process never initialised HIP
LAUNCHER_ENV = "MLOP_LAUNCHER_INFO"
WARMUP_STARTED = False  # set by server.start_hip_warmup (never in a launcher)


def kfd_open() -> bool:
    """True when this process holds a /dev/kfd descriptor (the HIP runtime opened the GPU)."""
    try:
        fds = os.listdir("/proc/self/fd")
    except OSError:
        return False
    for fd in fds:
        try:
            if os.readlink(f"/proc/self/fd/{fd}") == "/dev/kfd":
                return True
        except OSError:
            continue
    return False


def visible_gpu_count(topology: str = "/sys/class/kfd/kfd/topology/nodes", dev_dir: str = "/dev/dri") -> int:
    """GPUs this process could open, WITHOUT loading or initialising any HIP / torch code (a
    launcher must not touch the GPU before its rank children exist):

      * ``HIP_VISIBLE_DEVICES`` / ``ROCR_VISIBLE_DEVICES`` / ``CUDA_VISIBLE_DEVICES``: their count;
      * else the KFD topology: nodes with SIMDs (GPUs; CPU nodes report ``simd_count 0``) whose
        render node ``/dev/dri/renderD<drm_render_minor>`` exists and is read/writable here (a
        container sees only the render nodes of the GPUs it was given).
    0 when neither says anything (no GPU, no amdgpu driver)."""
    for var in ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        vis = os.environ.get(var)
        if vis is not None and vis.strip() != "":
            return len([x for x in vis.split(",") if x.strip() and x.strip() != "-1"])
    n = 0
    try:
        nodes = os.listdir(topology)
    except OSError:
        return 0
    for node in nodes:
        props = {}
        try:
            with open(os.path.join(topology, node, "properties")) as f:
                for line in f:
                    k, _, v = line.strip().partition(" ")
                    props[k] = v
        except OSError:
            continue
        try:
            if int(props.get("simd_count", "0")) <= 0:
                continue
            minor = int(props.get("drm_render_minor", "-1"))
        except ValueError:
            continue
        dev = os.path.join(dev_dir, f"renderD{minor}")
        if minor >= 0 and os.access(dev, os.R_OK | os.W_OK):
            n += 1
    return n


def _int_flag(argv: list[str], name: str) -> int:
    v = 1
    for i, a in enumerate(argv):
        if a == name and i + 1 < len(argv):
            v = int(argv[i + 1])
        elif a.startswith(name + "="):
            v = int(a.split("=", 1)[1])
    return v


def share_gpu_requested(argv: list[str], env=None) -> bool:
    env = os.environ if env is None else env
    return "--share-gpu" in argv or env.get("MLOP_SHARE_GPU", "0") not in ("", "0", "false")


def launcher_degree(argv: list[str], env=None) -> int:
    """N > 1 when this process must launch N ranks (``--tp N`` / ``--ep N`` and no WORLD_SIZE:
    not already a rank), else 1.  Pure argv / env parsing: safe before any import of torch."""
    env = os.environ if env is None else env
    if "WORLD_SIZE" in env:
        return 1
    try:
        return max(_int_flag(argv, "--tp"), _int_flag(argv, "--ep"), 1)
    except ValueError:
        return 1  # malformed: the server's argparse reports it


def launch_ranks(n: int, argv: list[str], share_gpu: bool | None = None) -> int:
    if share_gpu is None:
        share_gpu = share_gpu_requested(argv)
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    info = {"pid": os.getpid(), "ranks": n, "share_gpu": bool(share_gpu),
            # modules that would mean the launcher could have touched the GPU
            "torch_imported": "torch" in sys.modules,
            "hip_warmup_started": WARMUP_STARTED, "kfd_open": kfd_open()}
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK="0" if share_gpu else str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), MASTER_ADDR=os.environ.get("MASTER_ADDR", "127.0.0.1"),
                   MASTER_PORT=str(port), HSA_ENABLE_IPC_MODE_LEGACY="0", **{LAUNCHER_ENV: json.dumps(info)})
        if share_gpu:
            env["MLOP_SHARE_GPU"] = "1"
            env.setdefault("MLOP_CUSTOM_AR", "force")  # K15 / IPC kernels over the gloo group
        procs.append(subprocess.Popen([sys.executable, "-m", "mlopamd.runtime.server", *argv], env=env))

    def forward(sig, _frame):
        for p in procs:
            if p.poll() is None:
                p.send_signal(sig)

    signal.signal(signal.SIGTERM, forward)
    signal.signal(signal.SIGINT, forward)
    rc = 0
    try:
        while True:
            done = [p for p in procs if p.poll() is not None]
            if done:
                rc = next((p.returncode for p in done if p.returncode), 0)
                break
            time.sleep(0.2)
    finally:
        for p in procs:
            if p.poll() is None:
                p.terminate()
                try:
                    p.wait(timeout=10 if p is procs[0] else 3)
                except subprocess.TimeoutExpired:
                    p.kill()
    return rc
