"""Llama-3 decoder (8B / 70B shapes) for the serving runtime.

Flattened ragged batches (every scheduled token of every sequence in one
[T, H] matrix, vLLM-style) so prefill chunks and decode tokens share one
forward.  Per layer:

  add_rmsnorm -> QKV GEMM + RoPE + paged KV write (one kernel for M > 256) -> paged_attention
  -> O GEMM -> [TP all-reduce] -> add_rmsnorm -> gate_up GEMM -> silu_mul
  -> down GEMM -> [TP all-reduce]

Tensor parallel (Megatron): column-parallel QKV / gate_up, row-parallel O /
down, vocab-parallel embedding and LM head (2 all-reduces per layer over RCCL).
Weights are random-initialised on device (no checkpoints in this environment).
"""
from __future__ import annotations

import torch

from .. import ops
from ..parallel.comm import ParallelState, single
from ..parallel.overlap import row_parallel_add_norm
from .config import ModelConfig
from .layers import init_norm, init_weight, linear, rope_table




class LlamaModel:
    def __init__(self, cfg: ModelConfig, device="cuda", dtype=torch.bfloat16,
                 pstate: ParallelState | None = None, seed: int = 0):
        self.cfg = cfg
        self.device = torch.device(device)
        self.dtype = dtype
        self.ps = pstate or single()
        tp, r = self.ps.tp_size, self.ps.tp_rank
        assert cfg.num_heads % tp == 0, "q heads must divide by TP"
        assert cfg.intermediate_size % tp == 0 and cfg.vocab_size % tp == 0
        self.n_q = cfg.num_heads // tp
        # kv heads: sharded when tp <= Hkv, replicated otherwise
        self.n_kv = max(1, cfg.num_kv_heads // tp)
        self.inter = cfg.intermediate_size // tp
        self.vocab_local = cfg.vocab_size // tp
        self.vocab_start = r * self.vocab_local
        D, H = cfg.head_dim, cfg.hidden_size
        gen = torch.Generator(device=self.device)
        gen.manual_seed(seed * 1000 + r)
        w = lambda *s: init_weight(s, self.device, dtype, gen=gen)  # noqa: E731
        self.embed = w(self.vocab_local, H)
        self.layers = []
        for _ in range(cfg.num_layers):
            layer = {
                "in_norm": init_norm(H, self.device, dtype),
                "post_norm": init_norm(H, self.device, dtype),
                "qkv": w((self.n_q + 2 * self.n_kv) * D, H),
                "o": w(H, self.n_q * D),
            }
            layer.update(self._init_mlp(w))
            self.layers.append(layer)
        self.final_norm = init_norm(H, self.device, dtype)
        self.lm_head = self.embed if cfg.tie_embeddings else w(self.vocab_local, H)
        self.cos_sin = rope_table(D, cfg.max_position, cfg.rope_theta, cfg.rope_scaling, self.device)
        # in_norm / post_norm weights all ones (random init, or after fold_norms()): the large-M
        # TP=1 forward may then run the norm chain (ops.gemm_res_ss / gemm_rs)
        self.unit_norms = True

    # ---------------------------------------------------------- sharding --
    @torch.no_grad()
    def load_shard_from(self, full: "LlamaModel") -> "LlamaModel":
        """Copy this rank's TP shard out of a full (TP=1) model with the same config
        (checkpoint-style loading; also how the TP tests compare against TP=1)."""
        cfg, tp, r = self.cfg, self.ps.tp_size, self.ps.tp_rank
        D = cfg.head_dim
        kv_r = r * self.n_kv if tp <= cfg.num_kv_heads else (r * cfg.num_kv_heads) // tp
        qs = slice(r * self.n_q * D, (r + 1) * self.n_q * D)
        ks = slice(kv_r * D, (kv_r + self.n_kv) * D)
        vs = self.vocab_start, self.vocab_start + self.vocab_local
        dev = self.device

        def cp(dst, src):
            dst.copy_(src.to(dev, dst.dtype))

        cp(self.embed, full.embed[vs[0]:vs[1]])
        for L, F in zip(self.layers, full.layers):
            q, k, v = F["qkv"].split([cfg.q_size, cfg.kv_size, cfg.kv_size], 0)
            cp(L["qkv"], torch.cat([q[qs], k[ks], v[ks]], 0))
            cp(L["o"], F["o"][:, qs])
            cp(L["in_norm"], F["in_norm"])
            cp(L["post_norm"], F["post_norm"])
            self._shard_mlp(L, F)
        cp(self.final_norm, full.final_norm)
        if self.lm_head is not self.embed:
            cp(self.lm_head, full.lm_head[vs[0]:vs[1]])
        self.unit_norms = all(bool((L[k] == 1).all()) for L in self.layers for k in ("in_norm", "post_norm"))
        return self

    @torch.no_grad()
    def fold_norms(self) -> "LlamaModel":
        """Fold each RMSNorm weight into the projection that consumes it (in_norm -> qkv,
        post_norm -> gate_up: W[:, k] *= g[k]) and set the norm weights to ones, so the large-M
        forward can apply the normalisation as a per-row factor after the GEMM (norm chain).
        The same function up to the bf16 rounding of g * W."""
        for L in self.layers:
            for norm, proj in self._folds():
                g = L[norm].float()
                L[proj].copy_((L[proj].float() * g[None, :]).to(L[proj].dtype))
                L[norm].fill_(1)
        self.unit_norms = all(bool((L[k] == 1).all()) for L in self.layers for k in ("in_norm", "post_norm"))
        return self

    def _folds(self):
        return (("in_norm", "qkv"), ("post_norm", "gate_up"))

    def _shard_mlp(self, L, F):
        r, I = self.ps.tp_rank, self.inter
        L["gate_up"].copy_(F["gate_up"][2 * r * I:2 * (r + 1) * I].to(self.device, self.dtype))
        L["down"].copy_(F["down"][:, r * I:(r + 1) * I].to(self.device, self.dtype))

    # ---------------------------------------------------------------- MLP --
    def _init_mlp(self, w):
        # gate_up rows interleaved in groups of 16 (gate, up, gate, up, ...): the
        # GEMM's SiLU-mul epilogue then sees matching columns in one tile
        H = self.cfg.hidden_size
        return {"gate_up": w(2 * self.inter, H), "down": w(H, self.inter)}

    def mlp(self, i: int, x: torch.Tensor) -> torch.Tensor:
        L = self.layers[i]
        act = ops.gemm(x, L["gate_up"], epi=ops.EPI_SILU_MUL)  # K1/K2 + fused K8
        return linear(act, L["down"])

    def mlp_add_norm(self, i, x, residual, next_norm, eps):
        """TP=1: MLP whose down projection also does residual += and the next norm."""
        L = self.layers[i]
        act = ops.gemm(x, L["gate_up"], epi=ops.EPI_SILU_MUL)
        return ops.gemm_add_rmsnorm(act, L["down"], residual, next_norm, eps)

    def attn_out_mlp(self, i, a, residual, next_norm, eps):
        """TP=1: O projection with the residual add + post-attention norm in its reduce
        pass, then the MLP block with the next add + norm in the down projection's."""
        x = ops.gemm_add_rmsnorm(a, self.layers[i]["o"], residual, self.layers[i]["post_norm"], eps)
        return self.mlp_add_norm(i, x, residual, next_norm, eps)

    # ------------------------------------------------------------ forward --
    def weight_tensors(self):
        yield self.embed
        for L in self.layers:
            yield from (v for v in L.values() if isinstance(v, torch.Tensor))
        yield self.final_norm
        if self.lm_head is not self.embed:
            yield self.lm_head

    def weight_bytes(self) -> int:
        return sum(t.numel() * t.element_size() for t in self.weight_tensors())

    def forward(self, ids: torch.Tensor, meta, kv) -> torch.Tensor:
        """ids [T] int64; meta: AttnMeta (positions/slots/tables); kv: KVCache.
        Returns the final-normed hidden states of every token [T, H]."""
        cfg, tp = self.cfg, self.ps.tp
        eps = cfg.rms_eps
        h = ops.embedding(ids, self.embed, self.vocab_start)
        tp.all_reduce(h)
        residual = h
        M = ids.shape[0]
        # TP > 1: the decode (GEMV) form only, its residual adds riding in the all-reduces
        dmax = ops.decode_chain_max_m()  # the GEMV (<= 4 rows) / weight-streaming MFMA (<= 64) forms
        chain = (tp.size == 1 or M <= dmax) and self._chain_ok(M)
        ss = None  # norm chain: x is None and ss holds the residual's row partials
        if chain and M <= dmax:
            # decode form: the QKV GEMV takes the embedding rows' factors itself (ss unused)
            x, ss = None, ops.ss_init(h, ops.ss_buffer(M, cfg.hidden_size, h.device))
        else:
            x = ops.rmsnorm(h, self.layers[0]["in_norm"], eps)
        for i, L in enumerate(self.layers):
            if ss is None:
                q = ops.qkv_rope_cache(x, L["qkv"], meta.positions, self.cos_sin, meta.slots, kv.k[i], kv.v[i],
                                       self.n_q)
            else:
                q = ops.qkv_rope_cache_rs(residual, L["qkv"], meta.positions, self.cos_sin, meta.slots, kv.k[i],
                                          kv.v[i], self.n_q, ss, eps)
            a = ops.paged_attention(q, kv.k[i], kv.v[i], meta)
            nxt = self.layers[i + 1]["in_norm"] if i + 1 < len(self.layers) else self.final_norm
            if chain and tp.size > 1:
                x, ss = self._chain_layer_tp(i, a.view(a.shape[0], -1), residual, i + 1 == len(self.layers), eps, ss)
                continue
            if chain:
                x, ss = self._chain_layer(i, a.view(a.shape[0], -1), residual, i + 1 == len(self.layers), eps)
                continue
            if tp.size == 1:
                x = self.attn_out_mlp(i, a.view(a.shape[0], -1), residual, nxt, eps)
                continue
            # row-parallel O / down: the all-reduce + add + RMSNorm of row chunk i run on the
            # communication stream under the GEMM of chunk i+1 (parallel/overlap.py)
            x = row_parallel_add_norm(a.view(a.shape[0], -1), L["o"], tp, residual, L["post_norm"], eps)
            x = self.mlp_row_parallel(i, x, residual, nxt, eps)
        return x

    def mlp_row_parallel(self, i, x, residual, next_norm, eps):
        """TP > 1: gate_up (column-parallel, SiLU-mul fused), then the row-parallel down
        projection with its all-reduce overlapped, + the next residual add / norm."""
        act = ops.gemm(x, self.layers[i]["gate_up"], epi=ops.EPI_SILU_MUL)
        return row_parallel_add_norm(act, self.layers[i]["down"], self.ps.tp, residual, next_norm, eps)

    # --------------------------------------------------------- norm chain --
    def _chain_ok(self, M: int) -> bool:
        """Large-M TP=1 layers without add + RMSNorm passes: every GEMM of the chain on the
        four-wave kernel (ops.norm_chain_ok) and unit norm weights (folded into qkv / gate_up)."""
        if not self.unit_norms or len(self.layers) < 1:
            return False
        cfg, H = self.cfg, self.cfg.hidden_size
        return ops.norm_chain_ok(M, H, ((self.layers[0]["qkv"].shape[0], H), (H, self.n_q * cfg.head_dim),
                                        (2 * self.inter, H), (H, self.inter)), device=self.device,
                                 epis=(ops.EPI_ROPE, ops.EPI_NONE, ops.EPI_SILU_MUL, ops.EPI_NONE))

    def _chain_layer(self, i, a, residual, last, eps):
        """O (+= residual, row partials), gate_up + SiLU on the row-scaled residual, down (+=
        residual, row partials; the last layer's down does the final add + RMSNorm instead).
        Returns (x, ss): x normalised hidden states (last layer) or None with the partials."""
        L = self.layers[i]
        M, H = residual.shape
        ss_post = ops.ss_buffer(M, H, residual.device)
        ops.gemm_res_ss(a, L["o"], residual, ss_post)
        act = ops.gemm_rs(residual, L["gate_up"], ss_post, eps, ops.EPI_SILU_MUL)
        if last:
            return ops.gemm_add_rmsnorm(act, L["down"], residual, self.final_norm, eps), None
        ss = ops.ss_buffer(M, H, residual.device)
        ops.gemm_res_ss(act, L["down"], residual, ss)
        return None, ss

    def _chain_layer_tp(self, i, a, residual, last, eps, ss):
        """Tensor-parallel decode chain (M <= decode_chain_max_m()): the row-parallel O / down partial sums are
        all-reduced AND added into the replicated residual in one launch (Group.all_reduce_add,
        K15), gate_up and the next QKV take their rows' RMSNorm factors from the residual chunks
        they stream (gemv.hip PRO_RS).  Two add + RMSNorm launches per layer fewer than
        row_parallel_add_norm.  ss: the torch reference's row sums (unused by the GPU GEMVs)."""
        L, tp = self.layers[i], self.ps.tp
        o = ops.gemm(a, L["o"])
        tp.all_reduce_add(o, residual)
        act = ops.gemm_rs(residual, L["gate_up"], ops.ss_init(residual, ss), eps, ops.EPI_SILU_MUL)
        d = ops.gemm(act, L["down"])
        tp.all_reduce_add(d, residual)
        if last:
            return ops.rmsnorm(residual, self.final_norm, eps), None
        return None, ops.ss_init(residual, ss)

    def logits_local(self, hidden: torch.Tensor) -> torch.Tensor:
        """[n, H] -> this rank's vocab shard of the logits [n, V/TP] (model dtype)."""
        return linear(hidden, self.lm_head)

    def logits(self, hidden: torch.Tensor) -> torch.Tensor:
        """[n, H] -> full-vocab logits [n, V] in the model dtype (bf16 on GPU: the
        greedy argmax reads them directly, the sampler upcasts), gathered over TP."""
        return self.ps.tp.all_gather(self.logits_local(hidden), dim=-1)
