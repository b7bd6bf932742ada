"""Token sampling (K10): greedy, temperature, top-k, top-p.

GPU path: the fused HIP kernel ``torch.ops.mlop.sample`` (per-row top-k select
+ softmax + top-p + inverse-CDF draw, no full-vocab sort).  Greedy batches use
the HIP argmax directly on the LM head's bf16 logits (no fp32 copy).  CPU path: the same semantics in plain torch (oracle for tests).
"""
from __future__ import annotations

from dataclasses import dataclass, field

import torch

from .. import ops


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


MAX_TOP_K = 1024  # candidates kept by the sampling kernel (top_k=0 with top_p<1 uses this many)


def sample_reference(logits: torch.Tensor, temps: torch.Tensor, top_k: torch.Tensor,
                     top_p: torch.Tensor, uniform: torch.Tensor) -> torch.Tensor:
    """Plain-torch sampler with the kernel's semantics.

    temps/top_k/top_p/uniform: [n]; rows with temp <= 0 are greedy.  Candidates:
    the top min(top_k or MAX_TOP_K, V) logits; probabilities = softmax(l / T)
    over them; top-p keeps the smallest prefix with mass >= p; the token is the
    first candidate whose cumulative (renormalised) mass exceeds u."""
    n, V = logits.shape
    out = torch.empty(n, dtype=torch.int64, device=logits.device)
    kmax = min(MAX_TOP_K, V)
    vals, idx = torch.topk(logits.float(), kmax, dim=-1)  # sorted desc
    for i in range(n):
        if float(temps[i]) <= 0.0:
            out[i] = idx[i, 0]
            continue
        k = int(top_k[i]) if int(top_k[i]) > 0 else kmax
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

    def __call__(self, logits: torch.Tensor, params: list[SamplingParams]) -> torch.Tensor:
        n = logits.shape[0]
        if getattr(params, "all_greedy", False) or all(p.greedy for p in params[:n]):
            return ops.argmax(logits) if logits.is_cuda else logits.argmax(-1)
        dev = logits.device
        logits = logits.float()  # the top-k / top-p kernel works on fp32 rows
        temps = torch.tensor([p.temperature for p in params[:n]], dtype=torch.float32)
        ks = torch.tensor([p.top_k for p in params[:n]], dtype=torch.int32)
        ps = torch.tensor([p.top_p for p in params[:n]], dtype=torch.float32)
        u = torch.rand(n, generator=self.gen, device=self.device, dtype=torch.float32)
        if logits.is_cuda:
            return ops.sample(logits, temps.to(dev, non_blocking=True), ks.to(dev, non_blocking=True),
                              ps.to(dev, non_blocking=True), u)
        return sample_reference(logits, temps, ks, ps, u)
