"""Mixtral-8x7B (sparse MoE, top-2 of 8 experts) on the Llama attention stack.

MoE block (SURVEY.md §2.5 K11-K14 + CL4):
  router GEMM -> fused softmax/top-k/renormalise (K11) -> expert-sorted
  permutation (K12) -> grouped GEMM over all experts in ONE launch (K13,
  gate_up + SiLU-mul, then down) -> weighted un-permute/combine (K14).

Expert parallel: with ``ep > 1`` each rank owns E/ep experts; routed token
rows travel to their expert's rank with an all-to-all (dispatch) and back
(combine) over RCCL, see ``mlopamd.parallel.moe``.  Attention stays TP.
"""
from __future__ import annotations

import torch

from .. import ops
from .layers import linear
from .llama import LlamaModel


class MixtralModel(LlamaModel):
    def _init_mlp(self, w):
        cfg = self.cfg
        E, H, I = cfg.num_experts, cfg.hidden_size, cfg.intermediate_size
        ep = self.ps.ep.size
        assert E % ep == 0, "experts must divide by EP size"
        self.n_local_experts = E // ep
        self.expert_start = self.ps.ep.rank * self.n_local_experts
        return {
            "router": w(E, H),
            "w13": w(self.n_local_experts, 2 * I, H),
            "w2": w(self.n_local_experts, H, I),
        }

    def _shard_mlp(self, L, F):
        e0, n = self.expert_start, self.n_local_experts
        L["router"].copy_(F["router"].to(self.device, self.dtype))
        L["w13"].copy_(F["w13"][e0:e0 + n].to(self.device, self.dtype))
        L["w2"].copy_(F["w2"][e0:e0 + n].to(self.device, self.dtype))

    def _folds(self):
        return (("in_norm", "qkv"),)  # post_norm feeds the router and the experts

    def _chain_ok(self, M: int) -> bool:
        return False  # the norm chain is the dense MLP's (gate_up / down on the four-wave kernel)

    def mlp(self, i: int, x: torch.Tensor) -> torch.Tensor:
        from ..parallel.moe import moe_forward

        L = self.layers[i]
        # TP attention (tokens replicated on the EP group): partial sums, summed by the
        # layer's TP all-reduce.  DP attention (tp == 1, ep > 1): all-to-all dispatch.
        mode = "alltoall" if (self.ps.ep.size > 1 and self.ps.tp.size == 1) else "allreduce"
        # all-to-all capacity: the group's agreed token count of this step (engine.EPSync)
        cap = getattr(self, "moe_capacity_tokens", None)
        return moe_forward(x, L["router"], L["w13"], L["w2"], self.cfg.top_k, self.ps.ep,
                           self.expert_start, self.n_local_experts, mode=mode,
                           cap_tokens=max(cap or 0, x.shape[0]))

    def mlp_row_parallel(self, i, x, residual, next_norm, eps):
        """TP > 1 (experts sharded over the TP ranks): each rank's partial MoE output, summed by
        the TP all-reduce, then the next residual add / norm."""
        m = self.mlp(i, x)
        self.ps.tp.all_reduce(m)
        return ops.add_rmsnorm(m, residual, next_norm, eps)

    def mlp_add_norm(self, i, x, residual, next_norm, eps):
        """TP = EP = 1: MoE block + the next residual add / norm (decode-size dispatch in one
        launch, combine fused into the norm: parallel.moe.moe_forward_add_norm)."""
        if self.ps.ep.size == 1:
            from ..parallel.moe import moe_forward_add_norm

            L = self.layers[i]
            return moe_forward_add_norm(x, L["router"], L["w13"], L["w2"], self.cfg.top_k, self.expert_start,
                                        self.n_local_experts, residual, next_norm, eps)
        return ops.add_rmsnorm(self.mlp(i, x), residual, next_norm, eps)

    def attn_out_mlp(self, i, a, residual, next_norm, eps):
        """TP = EP = 1 decode sizes: O projection GEMV, then ONE launch for residual add +
        post-attention RMSNorm + router + route + sort + gather (moe_dispatch_small's
        prologue), the two grouped GEMMs, and the combine fused into the next add + norm."""
        if self.ps.ep.size == 1 and a.is_cuda and a.shape[0] <= 16:
            from ..parallel.moe import moe_forward_add_norm

            L = self.layers[i]
            o = linear(a, L["o"])
            return moe_forward_add_norm(None, L["router"], L["w13"], L["w2"], self.cfg.top_k, self.expert_start,
                                        self.n_local_experts, residual, next_norm, eps, pre=(o, L["post_norm"]))
        return super().attn_out_mlp(i, a, residual, next_norm, eps)

