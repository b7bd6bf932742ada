"""Model architecture configs (random-init; shapes of the public checkpoints).

Llama-3 shapes: public HF ``config.json`` of meta-llama/Meta-Llama-3-8B / -70B
(rope_theta 5e5; Llama-3.1 adds the "llama3" rope scaling, kept optional here).
Mixtral-8x7B: transformers ``MixtralConfig`` defaults (SURVEY.md §2.5 model table).
"""
from __future__ import annotations

from dataclasses import asdict, dataclass, field, replace


@dataclass(frozen=True)
class ModelConfig:
    name: str
    vocab_size: int
    hidden_size: int
    intermediate_size: int
    num_layers: int
    num_heads: int
    num_kv_heads: int
    head_dim: int = 128
    rope_theta: float = 500000.0
    rms_eps: float = 1e-5
    max_position: int = 8192
    tie_embeddings: bool = False
    # MoE (Mixtral): 0 experts = dense MLP
    num_experts: int = 0
    top_k: int = 2
    rope_scaling: dict | None = field(default=None, hash=False, compare=False)
    eos_token_id: int = 128001
    # further end-of-sequence ids (HF eos_token_id lists, e.g. Llama-3.1-Instruct's
    # [128001, 128008, 128009]: <|eot_id|> must stop generation too)
    extra_eos_ids: tuple = field(default=(), hash=False, compare=False)

    @property
    def eos_ids(self) -> tuple:
        return (self.eos_token_id, *self.extra_eos_ids)

    @property
    def is_moe(self) -> bool:
        return self.num_experts > 0

    @property
    def q_size(self) -> int:
        return self.num_heads * self.head_dim

    @property
    def kv_size(self) -> int:
        return self.num_kv_heads * self.head_dim

    def num_params(self) -> int:
        H, I, V, L = self.hidden_size, self.intermediate_size, self.vocab_size, self.num_layers
        attn = H * (self.q_size + 2 * self.kv_size) + self.q_size * H
        mlp = 3 * H * I * (self.num_experts if self.is_moe else 1)
        router = H * self.num_experts if self.is_moe else 0
        norms = 2 * H
        emb = V * H * (1 if self.tie_embeddings else 2)
        return L * (attn + mlp + router + norms) + emb + H

    def active_params(self) -> int:
        if not self.is_moe:
            return self.num_params()
        dense = replace(self, num_experts=0)
        extra = self.num_layers * 3 * self.hidden_size * self.intermediate_size * (self.top_k - 1)
        return dense.num_params() + extra + self.num_layers * self.hidden_size * self.num_experts

    def weight_bytes(self, dtype_bytes: int = 2) -> int:
        return self.num_params() * dtype_bytes

    def kv_bytes_per_token(self, dtype_bytes: int = 2) -> int:
        return 2 * self.num_layers * self.kv_size * dtype_bytes

    def flops_per_token(self) -> int:
        """Matmul FLOPs of one forward token (2 * active params, attention excluded)."""
        return 2 * self.active_params()

    def to_dict(self) -> dict:
        return asdict(self)


LLAMA3_8B = ModelConfig(
    name="llama3-8b", vocab_size=128256, hidden_size=4096, intermediate_size=14336,
    num_layers=32, num_heads=32, num_kv_heads=8, rope_theta=500000.0, max_position=8192)

LLAMA3_70B = ModelConfig(
    name="llama3-70b", vocab_size=128256, hidden_size=8192, intermediate_size=28672,
    num_layers=80, num_heads=64, num_kv_heads=8, rope_theta=500000.0, max_position=8192)

# Llama-3.1: same shapes, 128k context through the "llama3" RoPE frequency scaling
# (public HF config.json of meta-llama/Llama-3.1-8B / -70B)
_LLAMA31_ROPE = {"rope_type": "llama3", "factor": 8.0, "low_freq_factor": 1.0, "high_freq_factor": 4.0,
                 "original_max_position_embeddings": 8192}
LLAMA31_8B = replace(LLAMA3_8B, name="llama3.1-8b", max_position=131072, rope_scaling=_LLAMA31_ROPE)
LLAMA31_70B = replace(LLAMA3_70B, name="llama3.1-70b", max_position=131072, rope_scaling=_LLAMA31_ROPE)

MIXTRAL_8X7B = ModelConfig(
    name="mixtral-8x7b", vocab_size=32000, hidden_size=4096, intermediate_size=14336,
    num_layers=32, num_heads=32, num_kv_heads=8, rope_theta=1e6, max_position=32768,
    num_experts=8, top_k=2, eos_token_id=2)

# tiny shapes for CPU unit tests / GPU smoke (same code paths: GQA 4, head_dim 128)
TINY_LLAMA = ModelConfig(
    name="tiny-llama", vocab_size=512, hidden_size=256, intermediate_size=512, num_layers=2,
    num_heads=4, num_kv_heads=1, max_position=2048, eos_token_id=1)

TINY_MIXTRAL = ModelConfig(
    name="tiny-mixtral", vocab_size=512, hidden_size=256, intermediate_size=256, num_layers=2,
    num_heads=4, num_kv_heads=1, max_position=2048, num_experts=4, top_k=2, eos_token_id=1)

# CPU rehearsals of the 8-rank bench (bench.py --gpus 8 over gloo): 8 q heads so TP = 8 shards them
# (the one kv head is replicated), 8 experts so EP = 8 gives every rank one
TINY_LLAMA_8H = replace(TINY_LLAMA, name="tiny-llama-8h", num_heads=8)
TINY_MIXTRAL_8E = replace(TINY_MIXTRAL, name="tiny-mixtral-8e", num_experts=8)

PRESETS = {c.name: c for c in (LLAMA3_8B, LLAMA3_70B, LLAMA31_8B, LLAMA31_70B, MIXTRAL_8X7B, TINY_LLAMA,
                                TINY_MIXTRAL, TINY_LLAMA_8H, TINY_MIXTRAL_8E)}
# accepted aliases (MLflow tags / CR annotations use HF-ish names)
ALIASES = {
    "meta-llama/Meta-Llama-3-8B": "llama3-8b", "llama-3-8b": "llama3-8b", "Llama-3-8B": "llama3-8b",
    "meta-llama/Meta-Llama-3-70B": "llama3-70b", "llama-3-70b": "llama3-70b", "Llama-3-70B": "llama3-70b",
    "meta-llama/Llama-3.1-8B": "llama3.1-8b", "meta-llama/Meta-Llama-3.1-8B": "llama3.1-8b",
    "meta-llama/Llama-3.1-70B": "llama3.1-70b", "meta-llama/Meta-Llama-3.1-70B": "llama3.1-70b",
    "mistralai/Mixtral-8x7B-v0.1": "mixtral-8x7b", "Mixtral-8x7B": "mixtral-8x7b",
}


def get_config(name: str, **overrides) -> ModelConfig:
    key = ALIASES.get(name, name)
    if key not in PRESETS:
        raise KeyError(f"unknown model '{name}' (known: {sorted(PRESETS)})")
    cfg = PRESETS[key]
    return replace(cfg, **overrides) if overrides else cfg
