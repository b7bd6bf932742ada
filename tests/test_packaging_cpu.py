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
