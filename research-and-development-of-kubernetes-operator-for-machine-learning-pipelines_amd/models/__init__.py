"""Model zoo: Llama-3 (8B / 70B) and Mixtral-8x7B (MoE), random-init bf16.

The configs import without torch (the operator image's placement planner reads them);
``build_model`` pulls in torch and the model code on first use."""
from __future__ import annotations

from .config import ModelConfig, get_config, PRESETS  # noqa: F401


def build_model(name_or_cfg, device="cuda", dtype=None, pstate=None, seed: int = 0):
    import torch

    dtype = torch.bfloat16 if dtype is None else dtype
    cfg = name_or_cfg if isinstance(name_or_cfg, ModelConfig) else get_config(name_or_cfg)
    if cfg.is_moe:
        from .mixtral import MixtralModel

        return MixtralModel(cfg, device=device, dtype=dtype, pstate=pstate, seed=seed)
    from .llama import LlamaModel

    return LlamaModel(cfg, device=device, dtype=dtype, pstate=pstate, seed=seed)
