"""Token sampling (K10): greedy, temperature, top-k, top-p.

GPU path: the fused HIP kernel ``torch.ops.mlop.sample`` (per-row top-k select
+ softmax + top-p + inverse-CDF draw, no full-vocab sort).  Greedy batches use
the HIP argmax directly on the LM head's bf16 logits (no fp32 copy).  CPU path: the same semantics in plain torch (oracle for tests).
"""
from __future__ import annotations

from dataclasses import dataclass, field

import torch

from .. import ops

I32_MAX = 2**31 - 1
# stop ids per request: bounded so every backend (single GPU, TP, the EP group's fixed control
# slot, ep_serving.py) accepts and rejects the same requests
MAX_STOP_IDS = 256


@dataclass
class SamplingParams:
    max_tokens: int = 128
    temperature: float = 0.0
    top_k: int = 0          # 0 = disabled
    top_p: float = 1.0
    ignore_eos: bool = False
    stop_token_ids: list = field(default_factory=list)
    seed: int | None = None

    @property
    def greedy(self) -> bool:
        return self.temperature <= 0.0

    def validate(self) -> "SamplingParams":
        """Raise ValueError for parameters no sampler can honour (a bad request fails alone)."""
        import math

        # every integer must survive the int32 / int64 tensors the sampler and the EP request
        # broadcast build from it: an unbounded value would raise inside the engine step and
        # take the whole serving loop down instead of this one request
        if not isinstance(self.max_tokens, int) or not 1 <= self.max_tokens <= I32_MAX:
            raise ValueError(f"max_tokens must be an int in [1, {I32_MAX}], got {self.max_tokens}")
        if not math.isfinite(float(self.temperature)) or self.temperature < 0:
            raise ValueError(f"temperature must be finite and >= 0, got {self.temperature}")
        if not isinstance(self.top_k, int) or self.top_k < 0:
            raise ValueError(f"top_k must be an int >= 0, got {self.top_k}")
        if self.top_k > I32_MAX:
            self.top_k = 0  # beyond any vocabulary: the same as no top-k bound (full vocabulary)
        if not (0.0 < float(self.top_p) <= 1.0):
            raise ValueError(f"top_p must be in (0, 1], got {self.top_p}")
        if len(self.stop_token_ids) > MAX_STOP_IDS:
            raise ValueError(f"at most {MAX_STOP_IDS} stop_token_ids, got {len(self.stop_token_ids)}")
        if any(not isinstance(t, int) or not 0 <= t <= I32_MAX for t in self.stop_token_ids):
            raise ValueError(f"stop_token_ids must be ints in [0, {I32_MAX}]")
        if self.seed is not None and (not isinstance(self.seed, int) or not 0 <= self.seed < 2**63):
            raise ValueError("seed must be an int in [0, 2**63)")
        return self


MAX_TOP_K = 1024  # candidates of the top-k kernel; top_k = 0 or > MAX_TOP_K draws from the whole vocabulary


def seeded_uniform(seed: int, index: int) -> float:
    """The uniform of draw ``index`` (the token's position in the request's output) of a request
    with ``SamplingParams.seed``: a splitmix64 hash of (seed, index), 24 bits, exact in fp32.
    Independent of the batch the request rides in, of preemption and of other requests."""
    z = (int(seed) * 0x9E3779B97F4A7C15 + (int(index) + 1) * 0xBF58476D1CE4E5B9) & 0xFFFFFFFFFFFFFFFF
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & 0xFFFFFFFFFFFFFFFF
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & 0xFFFFFFFFFFFFFFFF
    z ^= z >> 31
    return (z >> 40) / float(1 << 24)


def _sample_full_row(l: torch.Tensor, T: float, k: int, p: float, u: float) -> int:
    """One row without a candidate bound (top_k = 0 or > MAX_TOP_K), fp64: members = the top-k
    by value (ties at the k-th value all kept) or the whole vocabulary; nucleus = the smallest
    prefix of the members sorted by value (ties by index) whose softmax mass reaches p of the
    members' mass; the draw = inverse CDF over the nucleus in vocabulary order."""
    V = l.numel()
    l = l.double()
    member = torch.ones(V, dtype=torch.bool)
    if 0 < k < V:
        member = l >= torch.topk(l, k).values[-1]
    w = torch.exp((l - l.max()) / T) * member
    nucleus = member
    if p < 1.0:
        order = torch.sort(-l, stable=True).indices  # descending value, ties by index
        cum = torch.cumsum(w[order], 0)
        keep = min(int((cum < p * float(cum[-1])).sum()) + 1, int(member.sum()))
        nucleus = torch.zeros(V, dtype=torch.bool)
        nucleus[order[:keep]] = True
    c = torch.cumsum(w * nucleus, 0)
    return int(min(int((c <= u * float(c[-1])).sum()), V - 1))


def sample_reference(logits: torch.Tensor, temps: torch.Tensor, top_k: torch.Tensor,
                     top_p: torch.Tensor, uniform: torch.Tensor) -> torch.Tensor:
    """Plain-torch sampler with the kernels' semantics (sampling.hip).

    temps/top_k/top_p/uniform: [n]; rows with temp <= 0 are greedy (argmax, ties to the lowest
    index).  0 < top_k <= MAX_TOP_K: candidates = the top-k logits; probabilities =
    softmax(l / T) over them; top-p keeps the smallest prefix with mass >= p; the token is the
    first candidate whose cumulative (renormalised) mass exceeds u.  top_k = 0 (or larger than
    MAX_TOP_K): the softmax over the WHOLE vocabulary (``_sample_full_row``)."""
    n, V = logits.shape
    out = torch.empty(n, dtype=torch.int64, device=logits.device)
    kmax = min(MAX_TOP_K, V)
    lf = logits.float()
    vals, idx = torch.topk(lf, kmax, dim=-1)  # sorted desc
    for i in range(n):
        if float(temps[i]) <= 0.0:
            out[i] = lf[i].argmax()
            continue
        k = int(top_k[i])
        if k <= 0 or k > MAX_TOP_K:
            out[i] = _sample_full_row(lf[i].cpu(), float(temps[i]), k, float(top_p[i]), float(uniform[i]))
            continue
        k = min(k, kmax)
        v = vals[i, :k] / float(temps[i])
        p = torch.softmax(v, dim=-1)
        c = torch.cumsum(p, dim=-1)
        pp = float(top_p[i])
        if pp < 1.0:
            keep = int((c < pp).sum().item()) + 1
            keep = min(keep, k)
            p = p[:keep] / c[keep - 1]
            c = torch.cumsum(p, dim=-1)
        j = int((c <= float(uniform[i])).sum().item())
        j = min(j, c.numel() - 1)
        out[i] = idx[i, j]
    return out


class Sampler:
    def __init__(self, device, seed: int = 0):
        self.device = torch.device(device)
        self.gen = torch.Generator(device=self.device)
        self.gen.manual_seed(seed)

    def __call__(self, logits: torch.Tensor, params: list[SamplingParams], gen_index=None) -> torch.Tensor:
        """``gen_index``: per row, the position of this draw in its request's output (array, or a
        callable returning one; only consulted when a row has ``SamplingParams.seed``)."""
        n = logits.shape[0]
        if getattr(params, "all_greedy", False) or all(p.greedy for p in params[:n]):
            return ops.argmax(logits) if logits.is_cuda else logits.argmax(-1)
        dev = logits.device
        logits = logits.float()  # the top-k / top-p kernel works on fp32 rows
        rows = params[:n]
        temps = torch.tensor([p.temperature for p in rows], dtype=torch.float32)
        ks = torch.tensor([p.top_k for p in rows], dtype=torch.int32)
        ps = torch.tensor([p.top_p for p in rows], dtype=torch.float32)
        u = torch.rand(n, generator=self.gen, device=self.device, dtype=torch.float32)
        seeded = [i for i, p in enumerate(rows) if p.seed is not None and not p.greedy]
        if seeded:
            gi = gen_index() if callable(gen_index) else gen_index
            us = [seeded_uniform(rows[i].seed, int(gi[i]) if gi is not None else 0) for i in seeded]
            u[torch.tensor(seeded, device=self.device)] = torch.tensor(us, dtype=torch.float32).to(self.device)
        if logits.is_cuda:
            full = bool((((ks <= 0) | (ks > MAX_TOP_K)) & (temps > 0)).any())
            return ops.sample(logits, temps.to(dev, non_blocking=True), ks.to(dev, non_blocking=True),
                              ps.to(dev, non_blocking=True), u, full=full)
        return sample_reference(logits, temps, ks, ps, u)
