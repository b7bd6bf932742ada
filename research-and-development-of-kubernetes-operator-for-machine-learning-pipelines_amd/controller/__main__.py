"""Operator CLI.

  python -m mlopamd.controller run [--namespace NS | --all-namespaces]
      the operator against a real cluster (in-cluster SA or kubeconfig), MLflow
      REST (MLFLOW_TRACKING_URI), Prometheus (MLOP_PROMETHEUS_URL); /healthz + /metrics on :8080
  python -m mlopamd.controller demo [--steps N]
      BASELINE config 1 end to end on CPU: sqlite MLflow with an sklearn-iris
      model, MlflowModel CR -> SeldonDeployment -> runtime process (V2) ->
      weighted router -> predictions; then v2 canary to 100 %.
  python -m mlopamd.controller plan --model llama3-70b [--tp 8]
      HBM-aware placement for 288 GB MI355X.
  python -m mlopamd.controller manifests
      print the install manifests (namespace, CRD, RBAC, operator Deployment).
"""
from __future__ import annotations

import argparse
import asyncio
import json
import logging
import sys

from .crd import MANIFESTS, OperatorSettings


async def run_operator(namespace: str | None, port: int):
    from .app import OperatorMetrics, make_operator, serve_health
    from .clock import RealClock
    from .kube import RestKube
    from .mlflow import MlflowRestClient
    from .prometheus import PromClient

    settings = OperatorSettings.from_env()
    metrics = OperatorMetrics()
    kube = RestKube.from_environment()
    op, _ = make_operator(kube, MlflowRestClient(), PromClient(settings.prometheus_url), RealClock(),
                          settings, namespace=namespace, metrics=metrics)
    await serve_health(metrics, port=port)
    await op.run()


def main(argv=None):
    logging.basicConfig(level=logging.INFO, format="%(asctime)s %(name)s %(levelname)s %(message)s")
    ap = argparse.ArgumentParser(prog="python -m mlopamd.controller", description=__doc__,
                                 formatter_class=argparse.RawDescriptionHelpFormatter)
    sub = ap.add_subparsers(dest="cmd", required=True)
    r = sub.add_parser("run")
    r.add_argument("--namespace", default=None)
    r.add_argument("--all-namespaces", action="store_true")
    r.add_argument("--port", type=int, default=8080)
    d = sub.add_parser("demo")
    d.add_argument("--requests", type=int, default=200)
    p = sub.add_parser("plan")
    p.add_argument("--model", default="llama3-8b")
    p.add_argument("--tp", type=int, default=None)
    p.add_argument("--max-model-len", type=int, default=4096)
    p.add_argument("--max-num-seqs", type=int, default=256)
    sub.add_parser("manifests")
    a = ap.parse_args(argv)
    if a.cmd == "run":
        asyncio.run(run_operator(None if a.all_namespaces else a.namespace, a.port))
    elif a.cmd == "demo":
        from .demo import run_demo

        print(json.dumps(asyncio.run(run_demo(a.requests)), indent=2))
    elif a.cmd == "plan":
        from .placement import plan

        print(json.dumps(plan(a.model, a.max_model_len, a.max_num_seqs, requested_tp=a.tp).to_dict(), indent=2))
    elif a.cmd == "manifests":
        for f in ("namespace.yaml", "crd.yaml", "rbac.yaml", "operator-deployment.yaml"):
            sys.stdout.write((MANIFESTS / f).read_text() + "\n---\n")


if __name__ == "__main__":
    main()
