"""Paged KV cache (G5) sized for 288 GB of HBM3E per GPU.

Device side: one K and one V tensor per layer, pages of 16 tokens:
  k[layer] : [num_blocks, Hkv, 16, D]   (token-major: A operand of S^T = K.Q^T)
  v[layer] : [num_blocks, Hkv, D, 16]   (dim-major:  A operand of O^T = V^T.P^T)
allocated ZEROED once (the attention kernel relies on finite unused slots).

Host side: ``BlockAllocator`` hands out page ids (free-list, O(1) alloc/free).
"""
from __future__ import annotations

import time

import torch

BLOCK_SIZE = 16


def _sync(device) -> None:
    if torch.device(device).type == "cuda":
        torch.cuda.synchronize(device)


class KVCache:
    def __init__(self, num_layers: int, num_blocks: int, num_kv_heads: int, head_dim: int,
                 device, dtype=torch.bfloat16):
        self.num_layers, self.num_blocks = num_layers, num_blocks
        self.num_kv_heads, self.head_dim = num_kv_heads, head_dim
        t0 = time.perf_counter()
        self.k_all = torch.empty(num_layers, num_blocks, num_kv_heads, BLOCK_SIZE, head_dim,
                                 device=device, dtype=dtype)
        self.v_all = torch.empty(num_layers, num_blocks, num_kv_heads, head_dim, BLOCK_SIZE,
                                 device=device, dtype=dtype)
        _sync(device)
        t1 = time.perf_counter()
        self.k_all.zero_()
        self.v_all.zero_()
        _sync(device)
        self.timing_ms = {"kv_malloc_ms": int(1e3 * (t1 - t0)), "kv_zero_ms": int(1e3 * (time.perf_counter() - t1))}
        self.k = [self.k_all[i] for i in range(num_layers)]
        self.v = [self.v_all[i] for i in range(num_layers)]

    @staticmethod
    def bytes_per_block(num_layers, num_kv_heads, head_dim, dtype_bytes=2) -> int:
        return 2 * num_layers * num_kv_heads * BLOCK_SIZE * head_dim * dtype_bytes

    @property
    def nbytes(self) -> int:
        return (self.k_all.numel() + self.v_all.numel()) * self.k_all.element_size()


def blocks_for_budget(budget_bytes: int, num_layers, num_kv_heads, head_dim, dtype_bytes=2) -> int:
    return max(1, budget_bytes // KVCache.bytes_per_block(num_layers, num_kv_heads, head_dim, dtype_bytes))


class BlockAllocator:
    """Free-list page allocator.  Block 0 is reserved as the always-valid
    'null page' that padded block-table entries point at."""

    def __init__(self, num_blocks: int):
        if num_blocks < 2:
            raise ValueError("need at least 2 KV blocks")
        self.num_blocks = num_blocks
        self._free = list(range(num_blocks - 1, 0, -1))  # pop() yields 1, 2, ...

    @property
    def num_free(self) -> int:
        return len(self._free)

    def can_allocate(self, n: int) -> bool:
        return n <= len(self._free)

    def allocate(self, n: int) -> list[int]:
        if n > len(self._free):
            raise MemoryError(f"KV cache exhausted: want {n}, free {len(self._free)}")
        out = self._free[-n:] if n else []
        del self._free[len(self._free) - n:]
        return out[::-1]

    def free(self, blocks) -> None:
        self._free.extend(reversed(list(blocks)))

    def usage(self) -> float:
        return 1.0 - len(self._free) / (self.num_blocks - 1)


def blocks_needed(num_tokens: int) -> int:
    return (num_tokens + BLOCK_SIZE - 1) // BLOCK_SIZE
