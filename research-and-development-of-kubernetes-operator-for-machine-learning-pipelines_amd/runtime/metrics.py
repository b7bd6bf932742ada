"""Per-pod Prometheus metrics of the serving runtime.

Seldon-executor-compatible series (names and labels the reference's PromQL
filters on, mlflow_operator.py:367-410) so the canary gate works unchanged:

  seldon_api_executor_client_requests_seconds{_bucket,_sum,_count}
      {deployment_name, predictor_name, namespace, model_name, model_image, method, code, service}
  seldon_api_executor_server_requests_seconds{_bucket,_sum,_count}
      {... , code, service}   (service="predictions" | "feedback" | "generate")

plus the LLM runtime's own series (tokens, TTFT/TPOT histograms, running /
waiting sequences, KV-cache use) and GPU gauges from amd-smi / sysfs
(``gpu_metrics``), which the canary gate can also consume.
"""
from __future__ import annotations

import os

from prometheus_client import CollectorRegistry, Counter, Gauge, Histogram, generate_latest
from prometheus_client.core import GaugeMetricFamily

LAT_BUCKETS = (0.001, 0.0025, 0.005, 0.01, 0.025, 0.05, 0.1, 0.25, 0.5, 1.0, 2.5, 5.0, 10.0, 30.0, 60.0, 120.0)


class _EngineClock:
    """Collector of ``mlop_engine_clock_seconds`` + ``mlop_engine_tokens_at_clock`` from one
    tuple the engine thread replaces atomically (``RuntimeMetrics.mark_step``)."""

    def __init__(self, labels: dict):
        self.names = list(labels)
        self.values = [str(labels[k]) for k in self.names]
        self.snap = (0.0, 0.0)

    def collect(self):
        tokens, clock = self.snap
        g = GaugeMetricFamily("mlop_engine_clock_seconds", "Engine-thread clock at the end of the last step",
                              labels=self.names)
        g.add_metric(self.values, clock)
        yield g
        t = GaugeMetricFamily("mlop_engine_tokens_at_clock",
                              "Engine tokens emitted up to mlop_engine_clock_seconds (same snapshot)",
                              labels=self.names)
        t.add_metric(self.values, tokens)
        yield t


class RuntimeMetrics:
    def __init__(self, deployment: str | None = None, predictor: str | None = None,
                 namespace: str | None = None, model_name: str = "model", image: str = "mlopamd/runtime-rocm"):
        e = os.environ
        self.labels = {
            "deployment_name": deployment or e.get("SELDON_DEPLOYMENT_ID", "local"),
            "predictor_name": predictor or e.get("PREDICTOR_ID", "default"),
            "namespace": namespace or e.get("SELDON_NAMESPACE", "default"),
            "model_name": model_name,
            "model_image": image,
        }
        base = list(self.labels)
        self.registry = r = CollectorRegistry()
        self.client = Histogram("seldon_api_executor_client_requests_seconds",
                                "Latency of requests to the model (executor -> model)",
                                base + ["method", "code", "service"], buckets=LAT_BUCKETS, registry=r)
        self.server = Histogram("seldon_api_executor_server_requests_seconds",
                                "Latency of requests served by the executor",
                                base + ["method", "code", "service"], buckets=LAT_BUCKETS, registry=r)
        self.tokens_out = Counter("mlop_generated_tokens", "Generated tokens", base, registry=r)
        self.tokens_in = Counter("mlop_prompt_tokens", "Prompt tokens processed", base, registry=r)
        self.ttft = Histogram("mlop_time_to_first_token_seconds", "TTFT", base, buckets=LAT_BUCKETS, registry=r)
        self.tpot = Histogram("mlop_time_per_output_token_seconds", "TPOT", base,
                              buckets=(0.002, 0.005, 0.01, 0.02, 0.03, 0.05, 0.1, 0.2, 0.5, 1.0), registry=r)
        self.running = Gauge("mlop_num_requests_running", "Sequences decoding", base, registry=r)
        self.waiting = Gauge("mlop_num_requests_waiting", "Sequences queued", base, registry=r)
        self.kv_usage = Gauge("mlop_kv_cache_usage_ratio", "Fraction of KV pages in use", base, registry=r)
        self.kv_blocks = Gauge("mlop_kv_cache_blocks", "KV pages backed by memory (lazy arena: grows while serving)",
                               base, registry=r)
        self.kv_fill_failed = Gauge("mlop_kv_cache_fill_failed",
                                    "1 when the background KV fill could not back a chunk (serving continues "
                                    "on the pages already backed)", base, registry=r)
        self.ready = Gauge("mlop_ready", "1 when the model is loaded and graphs captured", base, registry=r)
        self.load_seconds = Gauge("mlop_model_load_seconds", "Start-up time to ready", base, registry=r)
        self.gpu_busy = Gauge("mlop_gpu_busy_percent", "GPU busy %", base + ["gpu"], registry=r)
        self.gpu_mem = Gauge("mlop_gpu_memory_used_bytes", "HBM used", base + ["gpu"], registry=r)
        self.gpu_mem_total = Gauge("mlop_gpu_memory_total_bytes", "HBM total", base + ["gpu"], registry=r)
        self.gpu_power = Gauge("mlop_gpu_power_watts", "Socket power", base + ["gpu"], registry=r)
        self.engine_steps = Counter("mlop_engine_steps", "Engine steps executed", base, registry=r)
        self.engine_tokens = Counter("mlop_engine_tokens", "Tokens emitted by engine steps", base, registry=r)
        # the engine thread's perf_counter at the end of its last step AND the token total at that
        # instant, exported from ONE snapshot (``mark_step``): a rate over two scrapes then needs
        # no client-side clock (the scrape's own latency on a busy event loop skewed a 2-3 s
        # window by up to ~12 %), and a scrape can never pair a new token count with an old clock
        # (two separately collected series could, by up to one step's tokens at each end)
        self._tok_total = 0.0
        self._clock = _EngineClock(self.labels)
        r.register(self._clock)
        self.kernel_time = Gauge("mlop_kernel_time_fraction", "rocprof kernel-time share per kernel class",
                                 base + ["kernel"], registry=r)

    def mark_step(self, tokens: int, now: float) -> None:
        """Engine thread, once per step: the step counters and the (token total, clock) pair."""
        self.engine_steps.labels(**self.labels).inc()
        if tokens:
            self.engine_tokens.labels(**self.labels).inc(tokens)
        self._tok_total += tokens
        self._clock.snap = (self._tok_total, now)  # one reference store: scrapes see a consistent pair

    def lv(self, **extra):
        return dict(self.labels, **extra)

    def observe_request(self, seconds: float, code: int = 200, service: str = "predictions", method: str = "POST"):
        kv = self.lv(method=method, code=str(code), service=service)
        self.server.labels(**kv).observe(seconds)
        if service != "feedback":
            self.client.labels(**kv).observe(seconds)

    def update_gpu(self, samples: list[dict]):
        for s in samples:
            g = str(s.get("gpu", 0))
            if s.get("busy_percent") is not None:
                self.gpu_busy.labels(**self.lv(gpu=g)).set(s["busy_percent"])
            if s.get("mem_used") is not None:
                self.gpu_mem.labels(**self.lv(gpu=g)).set(s["mem_used"])
            if s.get("mem_total") is not None:
                self.gpu_mem_total.labels(**self.lv(gpu=g)).set(s["mem_total"])
            if s.get("power_w") is not None:
                self.gpu_power.labels(**self.lv(gpu=g)).set(s["power_w"])

    def update_kernel_shares(self, shares: dict):
        """Per-class kernel-time shares (runtime.gpu_metrics.KernelTimeSampler)."""
        for k in ("gemm", "attention", "norm", "rope_cache", "moe", "sampling", "other"):
            self.kernel_time.labels(**self.lv(kernel=k)).set(float(shares.get(k, 0.0)))

    def exposition(self) -> bytes:
        return generate_latest(self.registry)
