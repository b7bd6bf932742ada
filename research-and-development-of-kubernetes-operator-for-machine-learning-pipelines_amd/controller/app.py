"""Operator assembly: handlers registered on the kopf-style framework.

Equivalent of the reference's module-level ``@kopf.on.create/update``
registration (mlflow_operator.py:26-27), but explicit and injectable: the
kube API, MLflow client, Prometheus client and clock are arguments, so the
same operator runs against a real cluster or the in-memory fakes.
"""
from __future__ import annotations

import logging

from prometheus_client import CollectorRegistry, Counter, Histogram, generate_latest

from .clock import RealClock
from .crd import GROUP, PLURAL, SELDON_GROUP, SELDON_PLURAL, SELDON_VERSION, VERSION, OperatorSettings
from .framework import Operator
from .reconciler import MlflowModelReconciler

log = logging.getLogger("mlopamd.operator")


class OperatorMetrics:
    """The operator's own metrics (the reference exported none)."""

    def __init__(self):
        self.registry = r = CollectorRegistry()
        self.reconcile = Histogram("mlop_operator_reconcile_seconds", "Reconcile pass latency", registry=r,
                                   buckets=(0.001, 0.005, 0.01, 0.05, 0.1, 0.5, 1, 5))
        self.cr_ready = Histogram("mlop_operator_version_to_ready_seconds",
                                  "New model version detected -> predictor ready", registry=r,
                                  buckets=(0.5, 1, 2, 5, 10, 30, 60, 120, 300, 600, 1800))
        self.events = Counter("mlop_operator_events", "K8s events emitted", ["reason"], registry=r)
        self.ready_samples: list[float] = []

    def observe_reconcile(self, s: float):
        self.reconcile.observe(s)

    def observe_ready(self, s: float):
        self.cr_ready.observe(s)
        self.ready_samples.append(s)

    def p50_ready(self) -> float | None:
        xs = sorted(self.ready_samples)
        return xs[len(xs) // 2] if xs else None

    def exposition(self) -> bytes:
        return generate_latest(self.registry)


def make_operator(kube, mlflow, prom, clock=None, settings: OperatorSettings | None = None,
                  namespace: str | None = None, metrics: OperatorMetrics | None = None):
    clock = clock or RealClock()
    op = Operator(kube, clock, namespace=namespace)
    rec = MlflowModelReconciler(kube, mlflow, prom, clock, op, settings or OperatorSettings(), metrics)
    orig_event = op.event

    async def counted_event(body, type, reason, message):  # noqa: A002
        if metrics:
            metrics.events.labels(reason=reason).inc()
        await orig_event(body, type, reason, message)

    op.event = counted_event

    @op.daemon(GROUP, VERSION, PLURAL)
    async def mlflowmodel_daemon(stopped, body, logger, **_):
        await rec.run(body, stopped, logger)

    @op.on_delete(GROUP, VERSION, PLURAL)
    async def mlflowmodel_deleted(name, namespace, logger, **_):
        # the SeldonDeployment is owned by the CR: garbage-collected by Kubernetes
        logger.info("[%s/%s] MlflowModel deleted; owned SeldonDeployment is garbage-collected", namespace, name)

    @op.event_handler(SELDON_GROUP, SELDON_VERSION, SELDON_PLURAL)
    async def seldon_changed(event_type, body, **_):
        for ref in body.get("metadata", {}).get("ownerReferences") or []:
            if ref.get("kind") == "MlflowModel":
                rec.kick(body["metadata"].get("namespace"), ref.get("name"))

    return op, rec


async def serve_health(op_metrics: OperatorMetrics, host: str = "0.0.0.0", port: int = 8080):
    """/healthz and /metrics of the operator pod."""
    from aiohttp import web

    app = web.Application()
    app.router.add_get("/healthz", lambda _: web.json_response({"ok": True}))
    app.router.add_get("/metrics", lambda _: web.Response(body=op_metrics.exposition(), content_type="text/plain"))
    runner = web.AppRunner(app)
    await runner.setup()
    await web.TCPSite(runner, host, port).start()
    return runner
