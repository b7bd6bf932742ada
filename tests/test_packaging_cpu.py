"""Deployability of the two images (docker/*.Dockerfile): the operator image carries no
torch, so every control-plane module (incl. the placement planner's model configs) must
import without it; every path the Dockerfiles COPY exists; the image tags the manifests
and the SD builder reference are the ones the Dockerfiles document."""
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

GUARD = r'''
import sys, builtins
real = builtins.__import__
def guard(name, *a, **k):
    if name == "torch" or name.startswith("torch."):
        raise ImportError("no torch in the operator image")
    return real(name, *a, **k)
builtins.__import__ = guard
sys.path.insert(0, %r)
import mlopamd.controller.app, mlopamd.controller.__main__, mlopamd.controller.reconciler
import mlopamd.controller.placement, mlopamd.controller.prometheus, mlopamd.controller.apiserver
from mlopamd.controller.placement import plan
from mlopamd.models.config import get_config
p = plan(get_config("llama3-70b"), gpus_per_node=8)
print("ok", p)
'''


def test_operator_imports_without_torch():
    r = subprocess.run([sys.executable, "-c", GUARD % ROOT], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and r.stdout.startswith("ok"), r.stderr[-3000:]


def _copies(path):
    txt = open(path).read()
    for m in re.finditer(r"^COPY\s+(.+)$", txt, re.M):
        *srcs, _dst = m.group(1).split()
        yield from srcs


def test_dockerfile_sources_exist():
    for f in ("runtime.Dockerfile", "operator.Dockerfile"):
        for src in _copies(os.path.join(ROOT, "docker", f)):
            assert os.path.exists(os.path.join(ROOT, src)), f"{f}: COPY source {src} missing"


def test_image_tags_match_manifests():
    from mlopamd.controller import seldon

    dep = open(os.path.join(ROOT, "manifests", "operator-deployment.yaml")).read()
    op_img = re.search(r"image:\s*(\S+)", dep).group(1)
    rt_img = re.search(r"MLOP_RUNTIME_IMAGE, value: \"([^\"]+)\"", dep).group(1)
    assert op_img in open(os.path.join(ROOT, "docker", "operator.Dockerfile")).read()
    assert rt_img in open(os.path.join(ROOT, "docker", "runtime.Dockerfile")).read()
    pred = seldon.build_predictor(1, "s3://mlflow/x", None, 100, runtime=seldon.RUNTIME_LLM)
    assert pred["componentSpecs"][0]["spec"]["containers"][0]["image"] == rt_img


ISOLATED = r"""
import sys, builtins
allowed = set(sys.argv[2].split(","))
real = builtins.__import__
def guard(name, globals=None, locals=None, fromlist=(), level=0):
    top = name.split(".")[0]
    if level == 0 and top not in sys.stdlib_module_names and top not in allowed and top != "mlopamd" \
            and not top.startswith("_"):
        raise ImportError(f"{name}: not installed in the operator image")
    return real(name, globals, locals, fromlist, level)
builtins.__import__ = guard
sys.path[:] = [sys.argv[1]] + [p for p in sys.path if p and "repo" not in p]
import mlopamd.controller.__main__, mlopamd.controller.app, mlopamd.controller.reconciler
import mlopamd.controller.apiserver, mlopamd.controller.kube, mlopamd.controller.mlflow
from mlopamd.controller.placement import plan
print("ok", plan("llama3-8b").tensorParallel)
"""


def test_operator_image_imports_from_copied_paths_only(tmp_path):
    """Build the operator image's file tree (exactly the Dockerfile's COPY sources) and import
    the operator from it with only the stdlib and the pip packages the Dockerfile installs."""
    import shutil

    df = os.path.join(ROOT, "docker", "operator.Dockerfile")
    txt = open(df).read()
    for m in re.finditer(r"^COPY\s+(.+)$", txt, re.M):
        *srcs, dst = m.group(1).split()
        for src in srcs:
            s_abs = os.path.join(ROOT, src)
            d_abs = os.path.join(tmp_path, dst) if dst.endswith("/") else os.path.join(tmp_path, dst)
            if os.path.isdir(s_abs):
                shutil.copytree(s_abs, d_abs, dirs_exist_ok=True,
                                ignore=shutil.ignore_patterns("__pycache__"))
            else:
                os.makedirs(d_abs if dst.endswith("/") else os.path.dirname(d_abs), exist_ok=True)
                shutil.copy(s_abs, d_abs)
    os.symlink(os.path.join(tmp_path, "research-and-development-of-kubernetes-operator-for-machine-learning-"
                                      "pipelines_amd"), os.path.join(tmp_path, "mlopamd"))
    pip = re.search(r"pip install --no-cache-dir ([^\n\\]+)", txt).group(1).split()
    mods = {"pyyaml": "yaml", "prometheus_client": "prometheus_client"}
    allowed = ",".join(mods.get(p, p) for p in pip)
    r = subprocess.run([sys.executable, "-c", ISOLATED, str(tmp_path), allowed], capture_output=True, text=True,
                       timeout=120, cwd=str(tmp_path))
    assert r.returncode == 0 and r.stdout.startswith("ok"), r.stderr[-3000:]


def test_stale_extension_is_refused(tmp_path):
    """ops.load() refuses a _C.so built from other sources (embedded source hash)."""
    from mlopamd.ops import build as b

    if not (b.OUT.exists()):
        import pytest

        pytest.skip("extension not built")
    code = (f"import sys; sys.path.insert(0, {ROOT!r})\n"
            "import mlopamd.ops.build as b\n"
            "b.source_hash = lambda: 'deadbeef'\n"
            "from mlopamd import ops\n"
            "try:\n    ops.load(build_if_missing=False)\nexcept ops.StaleExtension as e:\n    print('refused', e)\n")
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120)
    assert "refused" in r.stdout, r.stdout + r.stderr[-2000:]
    ok = subprocess.run([sys.executable, "-c", f"import sys; sys.path.insert(0, {ROOT!r})\n"
                         "from mlopamd import ops; print(ops.load(build_if_missing=False))"],
                        capture_output=True, text=True, timeout=120)
    assert ok.stdout.strip().endswith("True"), ok.stderr[-2000:]
