"""Prometheus side of the canary gate (reference C9/C11, mlflow_operator.py:363-460).

* ``PromClient`` — async ``/api/v1/query`` client (replaces prometheus_api_client); a
  backend that cannot answer raises ``MetricsUnavailable`` (the reference's client raised
  too and its handler crashed; here the canary pauses, see reconciler.canary_tick).
* ``get_model_metrics`` — the reference's SIX PromQL queries, verbatim shapes,
  per predictor: p95 latency, error count, error rate, mean latency, request
  count, feedback count.
* ``should_promote`` — the reference gate (relative p95 / error-rate / mean
  thresholds; any missing metric => no promotion) plus an optional absolute
  error-rate floor and extra GPU-side guards (rocprof/amd-smi series).
* ``MetricStore`` + ``evaluate`` — a small PromQL engine (selectors with
  =, !=, =~, !~ matchers, range vectors, rate/increase/irate, sum/avg/max/min
  [by|without], histogram_quantile, ``or on() vector(x)``, scalar arithmetic)
  so a local fake Prometheus answers exactly those queries over samples
  scraped from our runtime's /metrics (``Scraper``) or injected by tests.
"""
from __future__ import annotations

import asyncio
import bisect
import json
import math
import re
import time
from collections import defaultdict
from dataclasses import dataclass, field

# ------------------------------------------------------------ the gate --

LATENCY_HIST = "seldon_api_executor_client_requests_seconds"
SERVER_COUNT = "seldon_api_executor_server_requests_seconds_count"


def model_queries(deployment_name: str, predictor_name: str, namespace: str, window: int = 60) -> dict:
    """The six query strings of mlflow_operator.py:367-410."""
    sel = f'deployment_name="{deployment_name}", predictor_name="{predictor_name}", namespace="{namespace}"'
    w = f"[{window}s]"
    return {
        "latency_95th": f"histogram_quantile(0.95, sum(rate({LATENCY_HIST}_bucket{{{sel}}}{w})) by (le))",
        "error_responses": f'sum(increase({SERVER_COUNT}{{code!="200", {sel}}}{w})) or on() vector(0)',
        "total_responses": f"sum(increase({SERVER_COUNT}{{{sel}}}{w})) or on() vector(0)",
        "latency_sum": f"sum(increase({LATENCY_HIST}_sum{{{sel}}}{w})) or on() vector(0)",
        "latency_count": f"sum(increase({LATENCY_HIST}_count{{{sel}}}{w})) or on() vector(0)",
        "feedback": f'sum(increase({SERVER_COUNT}{{service="feedback", {sel}}}{w})) or on() vector(0)',
    }


TPOT_HIST = "mlop_time_per_output_token_seconds"
GPU_MEM = "mlop_gpu_memory_used_bytes"
GPU_POWER = "mlop_gpu_power_watts"


KERNEL_SHARE = "mlop_kernel_time_fraction"


def gpu_guard_queries(deployment_name: str, predictor_name: str, namespace: str, window: int = 60) -> dict:
    """Extra per-predictor series for the canary gate ("plus amd-smi /
    rocprof series"): mean time per output token from the LLM runtime's TPOT
    histogram, peak HBM use and mean socket power from its amd-smi gauges.
    A predictor that exports none of them (e.g. MLFLOW_SERVER / sklearn) yields
    None and the gate skips the guard."""
    sel = f'deployment_name="{deployment_name}", predictor_name="{predictor_name}", namespace="{namespace}"'
    w = f"[{window}s]"
    return {
        "tpot_avg": f"sum(increase({TPOT_HIST}_sum{{{sel}}}{w})) / sum(increase({TPOT_HIST}_count{{{sel}}}{w}))",
        "gpu_memory_used": f"max(max_over_time({GPU_MEM}{{{sel}}}{w}))",
        "gpu_power": f"avg(avg_over_time({GPU_POWER}{{{sel}}}{w}))",
        # in-process rocprof-style kernel-time shares (runtime.gpu_metrics.KernelTimeSampler):
        # a version whose attention or GEMM share of device time grew regressed on the GPU
        "attention_share": f'avg(avg_over_time({KERNEL_SHARE}{{{sel}, kernel="attention"}}{w}))',
        "gemm_share": f'avg(avg_over_time({KERNEL_SHARE}{{{sel}, kernel="gemm"}}{w}))',
    }


def _first(result):
    if not result:
        return None
    v = float(result[0]["value"][1])
    return None if math.isnan(v) else v


async def get_model_metrics(prom, deployment_name, predictor_name, namespace, elapsed_time=60,
                            extra_queries: dict | None = None) -> dict:
    """Same outputs as the reference's get_model_metrics, plus optional extra series
    (e.g. per-pod GPU counters) named by ``extra_queries``."""
    q = model_queries(deployment_name, predictor_name, namespace, elapsed_time)
    names = list(q)
    res = await asyncio.gather(*(prom.query(q[n]) for n in names))
    r = dict(zip(names, res))
    m = {"latency_95th": _first(r["latency_95th"])}
    m["error_responses"] = _first(r["error_responses"]) or 0.0
    total = _first(r["total_responses"]) or 0.0
    m["error_rate"] = m["error_responses"] / total if total > 0 else None
    lsum = _first(r["latency_sum"]) or 0.0
    lcnt = _first(r["latency_count"]) or 0.0
    m["latency_avg"] = lsum / lcnt if lcnt > 0 else None
    m["request_count"] = lcnt
    m["feedback_request_count"] = _first(r["feedback"]) or 0.0
    for name, query in (extra_queries or {}).items():
        m[name] = _first(await prom.query(query))
    return m


@dataclass
class GateResult:
    promote: bool
    reasons: list = field(default_factory=list)


def should_promote(new: dict, old: dict, thresholds: dict, error_rate_floor: float = 0.0,
                   extra_max_ratio: dict | None = None, logger=None,
                   latency_floor_s: float = 0.0) -> GateResult:
    """Reference gate (mlflow_operator.py:419-460): all of latency_95th, error_rate,
    latency_avg must exist for both; new <= old * (1 + threshold) for each.
    ``error_rate_floor``: also accept new error rate <= floor (the reference's
    relative test with a 0 baseline demands exactly 0 errors).  ``extra_max_ratio``:
    {metric: ratio} extra guards (e.g. GPU HBM use), skipped if either side is None.
    ``latency_floor_s``: latencies at or below this are always acceptable (relative
    tests on sub-millisecond latencies are noise; 0 reproduces the reference)."""
    reasons = []
    for k in ("latency_95th", "error_rate", "latency_avg"):
        if new.get(k) is None or old.get(k) is None:
            reasons.append(f"metric {k} not available")
    if reasons:
        if logger:
            logger.warning("gate: %s", "; ".join(reasons))
        return GateResult(False, reasons)
    ok = True
    for k in ("latency_95th", "latency_avg"):
        lim = old[k] * (1 + thresholds.get(k, 0.05))
        if new[k] > lim and new[k] > latency_floor_s:
            ok = False
            reasons.append(f"{k} {new[k]:.4g} > {lim:.4g}")
    lim = old["error_rate"] * (1 + thresholds.get("error_rate", 0.02))
    if new["error_rate"] > lim and new["error_rate"] > error_rate_floor:
        ok = False
        reasons.append(f"error_rate {new['error_rate']:.4g} > {lim:.4g}")
    for k, ratio in (extra_max_ratio or {}).items():
        if new.get(k) is not None and old.get(k) is not None and old[k] > 0 and new[k] > old[k] * ratio:
            ok = False
            reasons.append(f"{k} {new[k]:.4g} > {ratio} x {old[k]:.4g}")
    if logger:
        (logger.info if ok else logger.warning)("gate: %s", "promote" if ok else "; ".join(reasons))
    return GateResult(ok, reasons)


# ------------------------------------------------------------ client --

class MetricsUnavailable(Exception):
    """The metrics backend could not answer (unreachable, timeout, HTTP / query error).
    Distinct from an answer with no samples: the canary pauses on this instead of counting
    a failed gate attempt (a monitoring outage must not roll back a healthy version)."""


class PromClient:
    def __init__(self, url: str, timeout_s: float = 10.0):
        self.url = url.rstrip("/")
        self.timeout_s = timeout_s
        self._session = None

    async def query(self, q: str, at: float | None = None) -> list:
        import aiohttp

        if self._session is None or self._session.closed:
            self._session = aiohttp.ClientSession(timeout=aiohttp.ClientTimeout(total=self.timeout_s))
        params = {"query": q}
        if at is not None:
            params["time"] = str(at)
        try:
            async with self._session.get(f"{self.url}/api/v1/query", params=params) as r:
                d = await r.json(content_type=None)
        except Exception as e:  # noqa: BLE001 - transport / timeout / non-JSON body
            raise MetricsUnavailable(f"{type(e).__name__}: {e}"[:300]) from e
        if not isinstance(d, dict) or d.get("status") != "success":
            err = d.get("error") if isinstance(d, dict) else None
            raise MetricsUnavailable(f"query failed: {err or d!r}"[:300])
        res = d["data"]["result"]
        if d["data"].get("resultType") == "scalar":
            return [{"metric": {}, "value": res}]
        return res

    async def close(self):
        if self._session is not None:
            await self._session.close()


class LocalProm:
    """In-process query interface over a MetricStore (no HTTP)."""

    def __init__(self, store: "MetricStore", clock=None):
        self.store, self.clock = store, clock

    async def query(self, q: str, at: float | None = None) -> list:
        t = at if at is not None else (self.clock.now() if self.clock else time.time())
        return to_api(evaluate(q, self.store, t), t)

    async def close(self):
        pass


# ------------------------------------------------------------- storage --

class MetricStore:
    """Append-only sample store: series = (name, frozenset(labels)) -> [(t, v)]."""

    def __init__(self, retention_s: float = 3600.0):
        self.series: dict[tuple, list] = defaultdict(list)
        self.retention_s = retention_s

    def add(self, name: str, labels: dict, value: float, t: float):
        key = (name, frozenset(labels.items()))
        s = self.series[key]
        s.append((t, float(value)))
        if len(s) > 64 and s[0][0] < t - self.retention_s:
            cut = bisect.bisect_left(s, (t - self.retention_s, -math.inf))
            del s[:cut]

    def select(self, name: str, matchers: list):
        for (n, lbl), samples in self.series.items():
            if n != name:
                continue
            d = dict(lbl)
            if all(_match(d.get(k, ""), op, v) for k, op, v in matchers):
                yield d, samples

    def ingest_exposition(self, text: str, t: float, extra_labels: dict | None = None):
        """Ingest a Prometheus text-format scrape."""
        from prometheus_client.parser import text_string_to_metric_families

        for fam in text_string_to_metric_families(text):
            for s in fam.samples:
                labels = dict(s.labels)
                if extra_labels:
                    labels.update(extra_labels)
                self.add(s.name, labels, s.value, t)


def _match(val: str, op: str, pat: str) -> bool:
    if op == "=":
        return val == pat
    if op == "!=":
        return val != pat
    if op == "=~":
        return re.fullmatch(pat, val) is not None
    if op == "!~":
        return re.fullmatch(pat, val) is None
    raise ValueError(op)


# ---------------------------------------------------------- PromQL mini --

_TOK = re.compile(r"""\s*(?:
    (?P<num>\d+\.\d*|\.\d+|\d+(?:[eE][+-]?\d+)?)
  | (?P<dur>\[\s*\d+[smhd]\s*\])
  | (?P<str>"(?:[^"\\]|\\.)*")
  | (?P<op>=~|!~|!=|==|=|\(|\)|\{|\}|,|\+|-|\*|/)
  | (?P<id>[A-Za-z_:][A-Za-z0-9_:]*)
)""", re.X)


def _tokens(s: str):
    pos, out = 0, []
    while pos < len(s):
        m = _TOK.match(s, pos)
        if not m or m.end() == pos:
            if s[pos:].strip() == "":
                break
            raise ValueError(f"PromQL syntax error at {s[pos:pos + 20]!r}")
        pos = m.end()
        kind = m.lastgroup
        out.append((kind, m.group(kind)))
    return out


class _Parser:
    AGG = {"sum", "avg", "max", "min", "count"}

    def __init__(self, s):
        self.t = _tokens(s)
        self.i = 0

    def peek(self, k=0):
        return self.t[self.i + k] if self.i + k < len(self.t) else (None, None)

    def take(self, val=None):
        tok = self.peek()
        if val is not None and tok[1] != val:
            raise ValueError(f"expected {val!r}, got {tok[1]!r}")
        self.i += 1
        return tok

    def parse(self):
        e = self.expr()
        if self.i != len(self.t):
            raise ValueError(f"trailing tokens: {self.t[self.i:]}")
        return e

    def expr(self):
        left = self.term()
        while True:
            k, v = self.peek()
            if v in ("+", "-"):
                self.take()
                left = ("bin", v, left, self.term())
            elif k == "id" and v == "or":
                self.take()
                on = None
                if self.peek()[1] == "on":
                    self.take()
                    self.take("(")
                    on = self.labels_until_paren()
                left = ("or", left, self.term(), on)
            else:
                return left

    def term(self):
        left = self.atom()
        while self.peek()[1] in ("*", "/"):
            op = self.take()[1]
            left = ("bin", op, left, self.atom())
        return left

    def labels_until_paren(self):
        labels = []
        while self.peek()[1] != ")":
            k, v = self.take()
            if v != ",":
                labels.append(v)
        self.take(")")
        return labels

    def atom(self):
        k, v = self.peek()
        if k == "num":
            self.take()
            return ("num", float(v))
        if v == "(":
            self.take()
            e = self.expr()
            self.take(")")
            return e
        if k == "id":
            self.take()
            if v in self.AGG:
                by, without = None, None
                if self.peek()[1] in ("by", "without"):
                    mode = self.take()[1]
                    self.take("(")
                    lbl = self.labels_until_paren()
                    by, without = (lbl, None) if mode == "by" else (None, lbl)
                self.take("(")
                inner = self.expr()
                self.take(")")
                if self.peek()[1] in ("by", "without"):
                    mode = self.take()[1]
                    self.take("(")
                    lbl = self.labels_until_paren()
                    by, without = (lbl, None) if mode == "by" else (None, lbl)
                return ("agg", v, inner, by, without)
            if self.peek()[1] == "(":  # function call
                self.take("(")
                args = []
                while self.peek()[1] != ")":
                    args.append(self.expr())
                    if self.peek()[1] == ",":
                        self.take()
                self.take(")")
                return ("call", v, args)
            # selector
            matchers = []
            if self.peek()[1] == "{":
                self.take("{")
                while self.peek()[1] != "}":
                    lk, lname = self.take()
                    op = self.take()[1]
                    sk, sval = self.take()
                    matchers.append((lname, op, json.loads(sval)))
                    if self.peek()[1] == ",":
                        self.take()
                self.take("}")
            rng = None
            if self.peek()[0] == "dur":
                d = self.take()[1].strip("[] ")
                rng = float(d[:-1]) * {"s": 1, "m": 60, "h": 3600, "d": 86400}[d[-1]]
            return ("sel", v, matchers, rng)
        raise ValueError(f"unexpected token {v!r}")


def _window(samples, t, rng):
    lo = bisect.bisect_left(samples, (t - rng, -math.inf))
    hi = bisect.bisect_right(samples, (t, math.inf))
    return samples[lo:hi]


def _increase(w):
    if len(w) < 2:
        return None
    inc, prev = 0.0, w[0][1]
    for _, v in w[1:]:
        inc += v - prev if v >= prev else v  # counter reset
        prev = v
    return inc


def evaluate(q: str, store: MetricStore, t: float, lookback: float = 300.0):
    """Evaluate at time t.  Returns a float (scalar) or list[(labels, value)]."""
    return _eval(_Parser(q).parse(), store, t, lookback)


def _eval(node, store, t, lookback):
    kind = node[0]
    if kind == "num":
        return node[1]
    if kind == "sel":
        _, name, matchers, rng = node
        if rng is not None:
            return ("range", [(lbl, _window(s, t, rng), rng) for lbl, s in store.select(name, matchers)])
        out = []
        for lbl, s in store.select(name, matchers):
            w = _window(s, t, lookback)
            if w:
                out.append((dict(lbl, __name__=name), w[-1][1]))
        return out
    if kind == "call":
        fn, args = node[1], node[2]
        if fn in ("rate", "increase", "irate", "delta"):
            rv = _eval(args[0], store, t, lookback)
            assert isinstance(rv, tuple) and rv[0] == "range", f"{fn} needs a range vector"
            out = []
            for lbl, w, rng in rv[1]:
                if fn == "irate":
                    if len(w) >= 2 and w[-1][0] > w[-2][0]:
                        d = w[-1][1] - w[-2][1]
                        out.append((lbl, (d if d >= 0 else w[-1][1]) / (w[-1][0] - w[-2][0])))
                    continue
                inc = _increase(w) if fn != "delta" else (w[-1][1] - w[0][1] if len(w) >= 2 else None)
                if inc is None:
                    continue
                out.append((lbl, inc / rng if fn == "rate" else inc))
            return out
        if fn == "vector":
            return [({}, float(_eval(args[0], store, t, lookback)))]
        if fn == "scalar":
            v = _eval(args[0], store, t, lookback)
            return v[0][1] if isinstance(v, list) and len(v) == 1 else float("nan")
        if fn == "histogram_quantile":
            phi = float(_eval(args[0], store, t, lookback))
            vec = _eval(args[1], store, t, lookback)
            groups = defaultdict(list)
            for lbl, v in vec:
                if "le" not in lbl:
                    continue
                key = frozenset((k, x) for k, x in lbl.items() if k not in ("le", "__name__"))
                groups[key].append((float(lbl["le"]), v))
            return [(dict(k), _hq(phi, b)) for k, b in groups.items()]
        if fn in ("max_over_time", "min_over_time", "avg_over_time", "last_over_time", "sum_over_time",
                  "count_over_time"):
            rv = _eval(args[0], store, t, lookback)
            assert isinstance(rv, tuple) and rv[0] == "range", f"{fn} needs a range vector"
            agg = {"max_over_time": max, "min_over_time": min, "sum_over_time": sum, "count_over_time": len,
                   "avg_over_time": lambda xs: sum(xs) / len(xs), "last_over_time": lambda xs: xs[-1]}[fn]
            return [({k: x for k, x in lbl.items() if k != "__name__"}, float(agg([v for _, v in w])))
                    for lbl, w, _ in rv[1] if w]
        if fn in ("abs", "ceil", "floor", "sqrt", "exp", "ln"):
            f = {"abs": abs, "ceil": math.ceil, "floor": math.floor, "sqrt": math.sqrt,
                 "exp": math.exp, "ln": math.log}[fn]
            return [(l, f(v)) for l, v in _eval(args[0], store, t, lookback)]
        raise ValueError(f"unsupported function {fn}")
    if kind == "agg":
        _, op, inner, by, without = node
        vec = _eval(inner, store, t, lookback)
        groups = defaultdict(list)
        for lbl, v in vec:
            if by is not None:
                key = frozenset((k, lbl[k]) for k in by if k in lbl)
            elif without is not None:
                key = frozenset((k, x) for k, x in lbl.items() if k not in without and k != "__name__")
            else:
                key = frozenset()
            groups[key].append(v)
        f = {"sum": sum, "max": max, "min": min, "count": len,
             "avg": lambda xs: sum(xs) / len(xs)}[op]
        return [(dict(k), float(f(vs))) for k, vs in groups.items()]
    if kind == "or":
        _, a, b, on = node
        va, vb = _eval(a, store, t, lookback), _eval(b, store, t, lookback)
        if va:
            return va
        return vb
    if kind == "bin":
        _, op, a, b = node
        va, vb = _eval(a, store, t, lookback), _eval(b, store, t, lookback)
        f = {"+": lambda x, y: x + y, "-": lambda x, y: x - y, "*": lambda x, y: x * y,
             "/": lambda x, y: x / y if y != 0 else (math.nan if x == 0 else math.copysign(math.inf, x))}[op]
        if isinstance(va, float) and isinstance(vb, float):
            return f(va, vb)
        if isinstance(va, float):
            return [(l, f(va, v)) for l, v in vb]
        if isinstance(vb, float):
            return [(l, f(v, vb)) for l, v in va]
        idx = {frozenset((k, x) for k, x in l.items() if k != "__name__"): v for l, v in vb}
        out = []
        for l, v in va:
            key = frozenset((k, x) for k, x in l.items() if k != "__name__")
            if key in idx:
                out.append(({k: x for k, x in l.items() if k != "__name__"}, f(v, idx[key])))
        return out
    raise ValueError(kind)


def _hq(phi, buckets):
    """Prometheus histogram_quantile over (upper bound, cumulative count) pairs."""
    buckets = sorted(buckets)
    if not buckets or buckets[-1][0] != math.inf:
        return math.nan
    total = buckets[-1][1]
    if total <= 0:
        return math.nan
    rank = phi * total
    prev_ub, prev_c = 0.0, 0.0
    for ub, c in buckets:
        if c >= rank:
            if ub == math.inf:
                return prev_ub
            if c == prev_c:
                return ub
            return prev_ub + (ub - prev_ub) * (rank - prev_c) / (c - prev_c)
        prev_ub, prev_c = ub, c
    return buckets[-2][0] if len(buckets) > 1 else math.nan


def to_api(result, t) -> list:
    """Evaluator output -> Prometheus HTTP API 'result' list (vector form)."""
    if isinstance(result, float):
        return [{"metric": {}, "value": [t, repr(result)]}]
    if isinstance(result, tuple):
        raise ValueError("range vector at top level is not supported for instant queries")
    return [{"metric": {k: v for k, v in l.items() if k != "__name__"}, "value": [t, _fmt(v)]}
            for l, v in result]


def _fmt(v: float) -> str:
    if math.isnan(v):
        return "NaN"
    if math.isinf(v):
        return "+Inf" if v > 0 else "-Inf"
    return repr(float(v))


# ------------------------------------------------------------ fake server --

class Scraper:
    """Periodically scrape /metrics of registered targets into a MetricStore."""

    def __init__(self, store: MetricStore, clock=None, interval_s: float = 5.0):
        self.store, self.clock, self.interval_s = store, clock, interval_s
        self.targets: dict[str, dict] = {}  # url -> extra labels
        self._task = None

    def add_target(self, url: str, labels: dict | None = None):
        self.targets[url] = labels or {}

    def remove_target(self, url: str):
        self.targets.pop(url, None)

    async def scrape_once(self):
        import aiohttp

        now = self.clock.now() if self.clock else time.time()
        async with aiohttp.ClientSession(timeout=aiohttp.ClientTimeout(total=5)) as s:
            for url, labels in list(self.targets.items()):
                try:
                    async with s.get(url) as r:
                        self.store.ingest_exposition(await r.text(), now, labels)
                        self.store.add("up", dict(labels, instance=url), 1.0, now)
                except Exception:  # noqa: BLE001
                    self.store.add("up", dict(labels, instance=url), 0.0, now)

    async def run(self):
        while True:
            await self.scrape_once()
            await (self.clock.sleep(self.interval_s) if self.clock else asyncio.sleep(self.interval_s))

    def start(self):
        self._task = asyncio.get_running_loop().create_task(self.run())

    async def stop(self):
        if self._task:
            self._task.cancel()
            try:
                await self._task
            except (asyncio.CancelledError, Exception):  # noqa: BLE001
                pass


def prometheus_app(store: MetricStore, clock=None):
    from aiohttp import web

    async def query(req):
        q = req.query.get("query", "")
        t = float(req.query["time"]) if "time" in req.query else (clock.now() if clock else time.time())
        try:
            res = evaluate(q, store, t)
        except Exception as e:  # noqa: BLE001
            return web.json_response({"status": "error", "errorType": "bad_data", "error": str(e)}, status=400)
        if isinstance(res, float):
            return web.json_response({"status": "success", "data": {"resultType": "scalar", "result": [t, _fmt(res)]}})
        return web.json_response({"status": "success", "data": {"resultType": "vector", "result": to_api(res, t)}})

    app = web.Application()
    app.router.add_get("/api/v1/query", query)
    app.router.add_post("/api/v1/query", query)
    return app


async def serve_prometheus(store: MetricStore, host="127.0.0.1", port=0, clock=None):
    from aiohttp import web

    runner = web.AppRunner(prometheus_app(store, clock))
    await runner.setup()
    site = web.TCPSite(runner, host, port)
    await site.start()
    return runner, f"http://{host}:{site._server.sockets[0].getsockname()[1]}"  # noqa: SLF001
