"""HBM-aware placement (G2): size a predictor's model shards for 288 GB per MI355X.

Inputs: the model architecture (weights, KV bytes per token), the serving
targets (max concurrent sequences x max context), and the node (HBM per GPU,
GPUs per node).  Output: tensor-parallel / expert-parallel degree, GPUs to
request (``amd.com/gpu``), per-GPU weight and KV budgets and the resulting KV
token capacity.  The KV target is ``kv_target_fraction`` (default 0.5: the mean context of a
uniformly-aged batch) of max_num_seqs x max_model_len — the engine preempts
(recompute) on the rare tail instead of every replica paying for the worst
case.  Policy: the smallest power-of-two TP (dividing the head
counts) that fits weights + activation reserve + the KV target in
``utilization x HBM`` — bigger shards and fewer ranks mean fewer, larger
collectives over the point-to-point xGMI links.  An explicit TP request
wins if it fits; MoE models use EP over the same GPUs.
"""
from __future__ import annotations

from dataclasses import asdict, dataclass

from ..models.config import ModelConfig, get_config

GB = 1e9


@dataclass
class Placement:
    architecture: str
    tensorParallel: int
    expertParallel: int
    gpus: int
    weightGBPerGPU: float
    kvGBPerGPU: float
    kvTokenCapacity: int
    hbmGBPerGPU: float
    fits: bool
    reason: str = ""

    def to_dict(self) -> dict:
        return asdict(self)


def _valid_tp(cfg: ModelConfig, tp: int) -> bool:
    return cfg.num_heads % tp == 0 and cfg.intermediate_size % tp == 0 and cfg.vocab_size % tp == 0


def plan(arch: str | ModelConfig, max_model_len: int = 4096, max_num_seqs: int = 256,
         hbm_gb: float = 288.0, gpus_per_node: int = 8, utilization: float = 0.90,
         reserve_gb: float = 8.0, requested_tp: int | None = None, requested_ep: int | None = None,
         kv_target_fraction: float = 0.5, free_gpus: int | None = None) -> Placement:
    """``free_gpus``: GPUs the target node still has unallocated (reconciler.node_capacity);
    a placement needing more is returned with ``fits=False`` and the reason (the pod would
    stay Pending), whatever its HBM arithmetic says."""
    p = _plan(arch, max_model_len, max_num_seqs, hbm_gb, gpus_per_node, utilization, reserve_gb,
              requested_tp, requested_ep, kv_target_fraction)
    if free_gpus is not None and p.gpus > free_gpus:
        p.fits = False
        p.reason = (f"needs {p.gpus} GPUs (TP={p.tensorParallel}), the node has {free_gpus} of "
                    f"{gpus_per_node} amd.com/gpu free") + (f"; {p.reason}" if p.reason else "")
    return p


def _plan(arch, max_model_len, max_num_seqs, hbm_gb, gpus_per_node, utilization, reserve_gb, requested_tp,
          requested_ep, kv_target_fraction) -> Placement:
    cfg = arch if isinstance(arch, ModelConfig) else get_config(arch)
    usable = hbm_gb * utilization
    wbytes = cfg.weight_bytes()
    kv_tok = cfg.kv_bytes_per_token()
    kv_target = max_num_seqs * max_model_len * kv_tok * kv_target_fraction

    def evaluate(tp: int, ep: int) -> Placement:
        shards = max(tp, ep)
        w = wbytes / shards
        kv_split = min(tp, cfg.num_kv_heads)  # kv heads replicate beyond Hkv
        kv_per_gpu = kv_target / kv_split
        free = usable * GB - reserve_gb * GB - w
        cap = int(max(0.0, free) * kv_split / kv_tok)
        fits = free >= kv_per_gpu
        return Placement(cfg.name, tp, ep, shards, round(w / GB, 2), round(max(0.0, free) / GB, 2), cap,
                         hbm_gb, fits, "" if fits else
                         f"needs {round((w + kv_per_gpu) / GB + reserve_gb, 1)} GB/GPU > {round(usable, 1)}")

    if requested_tp:
        if not _valid_tp(cfg, requested_tp) or requested_tp > gpus_per_node:
            p = evaluate(1, 1)
            p.fits, p.reason = False, f"invalid tensorParallel={requested_tp} for {cfg.name}"
            return p
        ep = requested_ep or (requested_tp if cfg.is_moe else 1)
        return evaluate(requested_tp, ep)
    tp = 1
    while tp <= gpus_per_node:
        if _valid_tp(cfg, tp):
            ep = requested_ep or (tp if cfg.is_moe else 1)
            p = evaluate(tp, ep)
            if p.fits:
                return p
        tp *= 2
    p = evaluate(gpus_per_node, gpus_per_node if cfg.is_moe else 1)
    p.fits = False
    p.reason = p.reason or "does not fit one node"
    return p
