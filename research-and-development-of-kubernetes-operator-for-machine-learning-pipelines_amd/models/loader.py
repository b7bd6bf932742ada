"""Checkpoint loading: Hugging Face ``config.json`` + ``*.safetensors`` -> our model layout.

The operator hands a predictor its MLflow artifact URI (``s3://mlflow/<rel>``, reference
``mlflow_operator.py:125-127``).  When that artifact is reachable as a local directory
(``file://`` URI, a plain path, or ``s3://mlflow/<rel>`` under ``MLOP_ARTIFACT_ROOT``)
holding a Llama / Mixtral checkpoint in the HF layout, the runtime serves those weights;
otherwise it random-initialises the architecture named by the CR / MLflow tags (the
benchmark configuration: no checkpoints are downloadable here).

Layout mapping (HF name -> ours; TP sharding then reuses ``load_shard_from``):
  model.embed_tokens / lm_head / model.norm       -> embed / lm_head / final_norm
  self_attn.{q,k,v}_proj                         -> qkv  ([q; k; v] rows, rotate-half RoPE as HF)
  self_attn.o_proj                               -> o
  input_layernorm / post_attention_layernorm     -> in_norm / post_norm
  mlp.{gate,up}_proj                             -> gate_up (rows interleaved in groups of 16:
                                                    the GEMM's SiLU-mul epilogue layout)
  mlp.down_proj                                  -> down
  Mixtral: block_sparse_moe.gate | mlp.gate      -> router
           experts.{e}.w1 / w3 (legacy) or experts.gate_up_proj (fused) -> w13 (interleaved)
           experts.{e}.w2 or experts.down_proj   -> w2
Tensors are read lazily, one layer at a time (safetensors memory map), so a 141 GB
checkpoint never sits in host memory at once.
"""
from __future__ import annotations

import json
import os
from dataclasses import replace
from pathlib import Path

import torch

from .config import ModelConfig, PRESETS

_ARCH_NAMES = {"LlamaForCausalLM": "llama", "MixtralForCausalLM": "mixtral", "MistralForCausalLM": "llama"}


def resolve_model_dir(uri: str | None) -> Path | None:
    """Local checkpoint directory for a model URI, or None (serve random-init weights)."""
    if not uri:
        return None
    if uri.startswith("file://"):
        p = Path(uri[len("file://"):])
    elif uri.startswith("s3://"):
        root = os.environ.get("MLOP_ARTIFACT_ROOT")
        if not root:
            return None
        p = Path(root) / uri[len("s3://"):].split("/", 1)[-1]  # drop the bucket ("mlflow")
    elif "://" in uri:
        return None
    else:
        p = Path(uri)
    for cand in (p, p / "model", p / "checkpoint", p / "artifacts"):
        if (cand / "config.json").is_file() and any(cand.glob("*.safetensors")):
            return cand
    return None


def config_from_hf(d: dict, name: str | None = None) -> ModelConfig:
    """ModelConfig from an HF ``config.json`` dict (Llama / Mistral / Mixtral families)."""
    arch = (d.get("architectures") or ["LlamaForCausalLM"])[0]
    if arch not in _ARCH_NAMES:
        raise ValueError(f"unsupported checkpoint architecture {arch!r} (supported: {sorted(_ARCH_NAMES)})")
    if d.get("hidden_act", "silu") != "silu":
        raise ValueError(f"unsupported activation {d.get('hidden_act')!r}")
    H, nh = d["hidden_size"], d["num_attention_heads"]
    rp = d.get("rope_parameters") or {}
    theta = rp.get("rope_theta", d.get("rope_theta", 10000.0))
    scaling = d.get("rope_scaling")
    if scaling is None and rp.get("rope_type", "default") not in ("default", None):
        scaling = dict(rp)
    # settings this runtime cannot serve are REJECTED, never dropped (dropping any of them
    # gives wrong logits with no error)
    if scaling:
        rt = scaling.get("rope_type", scaling.get("type", "default"))
        if rt not in ("default", "llama3"):
            raise ValueError(f"unsupported rope_scaling type {rt!r} (supported: default, llama3)")
    max_pos = int(d.get("max_position_embeddings", 8192))
    sw = d.get("sliding_window")
    if sw is not None and d.get("use_sliding_window", True) and int(sw) < max_pos:
        raise ValueError(f"sliding_window={sw} < max_position_embeddings={max_pos}: "
                         "sliding-window attention is not implemented")
    for flag in ("attention_bias", "mlp_bias"):
        if d.get(flag):
            raise ValueError(f"{flag}=true is not supported (bias tensors are not loaded)")
    eos = d.get("eos_token_id", 2)
    eos_all = tuple(int(e) for e in eos) if isinstance(eos, list) else ((int(eos),) if eos is not None else (2,))
    eos = eos_all[0]
    return ModelConfig(
        name=name or d.get("_name_or_path") or arch, vocab_size=d["vocab_size"], hidden_size=H,
        intermediate_size=d["intermediate_size"], num_layers=d["num_hidden_layers"], num_heads=nh,
        num_kv_heads=d.get("num_key_value_heads") or nh, head_dim=d.get("head_dim") or H // nh,
        rope_theta=float(theta), rms_eps=float(d.get("rms_norm_eps", 1e-5)),
        max_position=max_pos,
        tie_embeddings=bool(d.get("tie_word_embeddings", False)),
        num_experts=int(d.get("num_local_experts", 0) or 0), top_k=int(d.get("num_experts_per_tok", 2)),
        rope_scaling=scaling, eos_token_id=int(eos), extra_eos_ids=eos_all[1:])


class _Tensors:
    """Name -> tensor over every ``*.safetensors`` shard of a directory (lazy, mmap)."""

    def __init__(self, path: Path):
        from safetensors import safe_open

        self._files = [safe_open(str(f), framework="pt") for f in sorted(path.glob("*.safetensors"))]
        self._where = {k: f for f in self._files for k in f.keys()}

    def has(self, k: str) -> bool:
        return k in self._where

    def get(self, k: str) -> torch.Tensor:
        if k not in self._where:
            raise KeyError(f"checkpoint has no tensor {k!r}")
        return self._where[k].get_tensor(k)


class _LazyLayer:
    """One decoder layer in our layout: every key is read (and re-laid-out) from the
    checkpoint when accessed, nothing is kept (one tensor in host memory at a time)."""

    def __init__(self, thunks: dict):
        self._thunks = thunks

    def __getitem__(self, k):
        return self._thunks[k]()

    def __contains__(self, k):
        return k in self._thunks


class HFWeights:
    """A TP=1 model's weights in our layout, read from an HF checkpoint (the ``full``
    argument of ``LlamaModel.load_shard_from``)."""

    def __init__(self, path: Path, cfg: ModelConfig):
        from ..ops import interleave_gate_up

        self.cfg = cfg
        t = _Tensors(path)
        self._t = t
        self.embed = t.get("model.embed_tokens.weight")
        self.final_norm = t.get("model.norm.weight")
        self.lm_head = t.get("lm_head.weight") if t.has("lm_head.weight") else self.embed

        def layer(i):
            p = f"model.layers.{i}."
            L = {"qkv": lambda: torch.cat([t.get(p + f"self_attn.{n}_proj.weight") for n in "qkv"], 0),
                 "o": lambda: t.get(p + "self_attn.o_proj.weight"),
                 "in_norm": lambda: t.get(p + "input_layernorm.weight"),
                 "post_norm": lambda: t.get(p + "post_attention_layernorm.weight")}
            if not cfg.is_moe:
                L["gate_up"] = lambda: interleave_gate_up(t.get(p + "mlp.gate_proj.weight"),
                                                          t.get(p + "mlp.up_proj.weight"))
                L["down"] = lambda: t.get(p + "mlp.down_proj.weight")
                return _LazyLayer(L)
            E, I = cfg.num_experts, cfg.intermediate_size
            if t.has(p + "block_sparse_moe.gate.weight"):  # legacy per-expert layout (save_pretrained)
                m = p + "block_sparse_moe."
                L["router"] = lambda: t.get(m + "gate.weight")
                L["w13"] = lambda: torch.stack([interleave_gate_up(t.get(m + f"experts.{e}.w1.weight"),
                                                                   t.get(m + f"experts.{e}.w3.weight"))
                                                for e in range(E)])
                L["w2"] = lambda: torch.stack([t.get(m + f"experts.{e}.w2.weight") for e in range(E)])
            else:  # fused expert tensors (transformers >= 5 module layout)
                m = p + "mlp."
                L["router"] = lambda: t.get(m + "gate.weight")

                def w13():
                    gu = t.get(m + "experts.gate_up_proj")  # [E, 2I, H]: gate rows then up rows
                    return torch.stack([interleave_gate_up(gu[e, :I], gu[e, I:]) for e in range(E)])

                L["w13"] = w13
                L["w2"] = lambda: t.get(m + "experts.down_proj")
            return _LazyLayer(L)

        self.layers = [layer(i) for i in range(cfg.num_layers)]


def load_pretrained(path: str | os.PathLike, device="cuda", dtype=torch.bfloat16, pstate=None,
                    name: str | None = None, fold_norms: bool = True):
    """Build our model for the checkpoint in ``path`` and copy its (TP-sharded) weights in."""
    from . import build_model

    path = Path(path)
    cfg = config_from_hf(json.loads((path / "config.json").read_text()), name=name or path.name)
    model = build_model(cfg, device=device, dtype=dtype, pstate=pstate)
    with torch.no_grad():
        model.load_shard_from(HFWeights(path, cfg))
    # checkpoints carry trained (non-unit) RMSNorm weights: fold them into the projections that
    # consume them so the large-M forward can run the norm chain (LlamaModel._chain_ok needs unit
    # norms).  The same function up to the bf16 rounding of g * W; fold_norms=False keeps them.
    if fold_norms:
        model.fold_norms()
    return model


def known_preset(cfg: ModelConfig) -> str | None:
    """Name of the preset with the same shapes (placement / reporting), if any."""
    for n, p in PRESETS.items():
        if replace(p, name=cfg.name, eos_token_id=cfg.eos_token_id, rope_scaling=cfg.rope_scaling,
                   max_position=cfg.max_position) == cfg:
            return n
    return None
