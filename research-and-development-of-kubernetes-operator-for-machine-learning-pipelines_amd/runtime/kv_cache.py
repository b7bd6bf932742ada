"""Paged KV cache (G5) sized for 288 GB of HBM3E per GPU.

Device side: one K and one V tensor per layer, pages of 16 tokens:
  k[layer] : [num_blocks, Hkv, 16, D]   (token-major: A operand of S^T = K.Q^T)
  v[layer] : [num_blocks, Hkv, 16, D]   (token-major too: a token's row is one contiguous
                                          store; attention.hip reads V^T out of LDS transposed)
zeroed before first use (the attention kernel relies on finite unused slots).

Two ways to back it:

* eager: two ``torch.empty`` + ``zero_`` (CPU, TP ranks, ``kv_cache.LAZY = False``);
* lazy (default on one GPU): ``ops/csrc/vmm.hip`` reserves the whole virtual range, backs
  and zeroes the first chunk of pages before the engine reports ready, and a native worker
  thread backs the rest while it serves.  A 134 GB hipMalloc waits 0.7-4.8 s for the
  driver to scrub memory another process just freed (profiles/r02_kv_lazy_map.md); backing
  4 GB first takes that wait off the CR -> ready path.  ``ready_blocks()`` says how many
  page ids are backed; the engine grows its ``BlockAllocator`` to it, so no page of an
  unbacked chunk is ever handed out.

Host side: ``BlockAllocator`` hands out page ids (free-list, O(1) alloc/free).
"""
from __future__ import annotations

import collections
import math
import os
import time

import numpy as np
import torch

BLOCK_SIZE = 16
CHUNK_BYTES_PER_REGION = 64 << 20   # lazy backing unit: 64 MB of each K / V layer tensor
INITIAL_BYTES = 4 << 30             # backed before ready (all layers, K and V)


def _sync(device) -> None:
    if torch.device(device).type == "cuda":
        torch.cuda.synchronize(device)


LAZY = True  # GPU pools lazily backed (tests flip it for the eager / lazy A/B)


def _lazy_default(device) -> bool:
    if torch.device(device).type != "cuda" or not LAZY:
        return False
    from .. import ops

    ops.load()
    idx = torch.device(device).index
    return bool(torch.ops.mlop.vmm_supported(torch.cuda.current_device() if idx is None else idx))


class KVCache:
    def __init__(self, num_layers: int, num_blocks: int, num_kv_heads: int, head_dim: int,
                 device, dtype=torch.bfloat16, lazy: bool | None = None, initial_blocks: int | None = None):
        self.num_layers, self.num_blocks = num_layers, num_blocks
        self.num_kv_heads, self.head_dim = num_kv_heads, head_dim
        self.device, self.dtype = torch.device(device), dtype
        self.lazy = _lazy_default(device) if lazy is None else lazy
        self.fill_failed = False  # a background chunk could not be backed: stop growing
        self._flat = None
        t0 = time.perf_counter()
        if self.lazy:
            self._init_lazy(initial_blocks)
            self.timing_ms = {"kv_malloc_ms": int(1e3 * (time.perf_counter() - t0)), "kv_zero_ms": 0}
        else:
            self.k_all = torch.empty(num_layers, num_blocks, num_kv_heads, BLOCK_SIZE, head_dim,
                                     device=device, dtype=dtype)
            self.v_all = torch.empty(num_layers, num_blocks, num_kv_heads, BLOCK_SIZE, head_dim,
                                     device=device, dtype=dtype)
            _sync(device)
            t1 = time.perf_counter()
            self.k_all.zero_()
            self.v_all.zero_()
            _sync(device)
            self.timing_ms = {"kv_malloc_ms": int(1e3 * (t1 - t0)), "kv_zero_ms": int(1e3 * (time.perf_counter() - t1))}
        self.k = [self.k_all[i] for i in range(num_layers)]
        self.v = [self.v_all[i] for i in range(num_layers)]

    def _init_lazy(self, initial_blocks):
        L, Hkv, D = self.num_layers, self.num_kv_heads, self.head_dim
        esz = torch.empty(0, dtype=self.dtype).element_size()
        page = Hkv * BLOCK_SIZE * D                      # elements of one page in one layer tensor
        page_bytes = page * esz
        idx = self.device.index if self.device.index is not None else torch.cuda.current_device()
        gran = int(torch.ops.mlop.vmm_granularity(idx))
        unit = gran // math.gcd(gran, page_bytes)          # pages per granule-aligned step
        cb = max(unit, (CHUNK_BYTES_PER_REGION // page_bytes) // unit * unit)
        self.chunk_blocks = cb
        self.n_chunks = -(-self.num_blocks // cb)
        chunk_bytes = cb * page_bytes
        region = self.n_chunks * chunk_bytes               # bytes of one layer's K (or V) tensor
        n_regions = 2 * L
        self._flat = torch.ops.mlop.vmm_arena(n_regions * region, idx)
        base = self._flat.view(self.dtype)
        rs = region // esz
        self.k_all = base.as_strided((L, self.num_blocks, Hkv, BLOCK_SIZE, D), (rs, page, BLOCK_SIZE * D, D, 1), 0)
        self.v_all = base.as_strided((L, self.num_blocks, Hkv, BLOCK_SIZE, D), (rs, page, BLOCK_SIZE * D, D, 1),
                                     L * rs)
        if initial_blocks is None:
            initial_blocks = max(2, INITIAL_BYTES // (n_regions * page_bytes))
        first = min(self.n_chunks, max(1, -(-initial_blocks // cb)))
        self._map_args = (region, n_regions, chunk_bytes)
        self._first = first
        self._filling = False
        if not torch.ops.mlop.vmm_map_chunks(self._flat, *self._map_args, 0, first, False):
            raise RuntimeError("KV arena: backing the first chunk failed")

    def start_background_fill(self) -> None:
        """Back the remaining chunks on a native worker thread.  Call it after any hipGraph
        capture: VMM calls from another thread would invalidate a global-mode capture."""
        if not self.lazy or self._filling or self._first >= self.n_chunks:
            return
        if not torch.ops.mlop.vmm_map_chunks(self._flat, *self._map_args, self._first,
                                             self.n_chunks - self._first, True):
            raise RuntimeError("KV arena: could not start the background backing thread")
        self._filling = True
        self._fill_t0 = time.perf_counter()

    def wait_ready(self, timeout_s: float = 300.0) -> dict:
        """Block until every page is backed (a lazy arena's background fill is done).
        Returns {"kv_fill_wait_ms": time spent here, "kv_fill_ms": fill start -> full}."""
        t0 = time.perf_counter()
        while self.ready_blocks() < self.num_blocks:
            if time.perf_counter() - t0 > timeout_s:
                raise TimeoutError(f"KV arena: {self.ready_blocks()} of {self.num_blocks} pages backed "
                                   f"after {timeout_s:.0f} s")
            time.sleep(0.005)
        t1 = time.perf_counter()
        start = getattr(self, "_fill_t0", None)
        return {"kv_fill_wait_ms": int(1e3 * (t1 - t0)),
                "kv_fill_ms": int(1e3 * (t1 - start)) if start is not None else 0}

    def ready_blocks(self) -> int:
        """Page ids [0, ready_blocks()) are backed and zeroed (all of them when eager)."""
        if not self.lazy:
            return self.num_blocks
        if torch.ops.mlop.vmm_error(self._flat) and not self.fill_failed:
            # e.g. another process took the memory freed before this arena's background fill
            # reached it: the chunks already backed stay valid and in use; the arena just
            # stops growing (the engine records it in stats / metrics)
            self.fill_failed = True
        return min(self.num_blocks, int(torch.ops.mlop.vmm_chunks_ready(self._flat)) * self.chunk_blocks)

    @staticmethod
    def bytes_per_block(num_layers, num_kv_heads, head_dim, dtype_bytes=2) -> int:
        return 2 * num_layers * num_kv_heads * BLOCK_SIZE * head_dim * dtype_bytes

    @property
    def nbytes(self) -> int:
        return 2 * self.num_layers * self.num_blocks * self.num_kv_heads * BLOCK_SIZE * self.head_dim * \
            self.k_all.element_size()


def blocks_for_budget(budget_bytes: int, num_layers, num_kv_heads, head_dim, dtype_bytes=2) -> int:
    return max(1, budget_bytes // KVCache.bytes_per_block(num_layers, num_kv_heads, head_dim, dtype_bytes))


class BlockAllocator:
    """Page allocator with reference counts and a prefix cache.

    Block 0 is reserved as the always-valid 'null page' that padded block-table
    entries point at.  ``available`` page ids (a prefix of [0, num_blocks)) may grow
    over time (``grow``: pages of a lazily backed KV arena becoming ready).

    Prefix caching (vLLM-style automatic prefix caching): a FULL page of computed
    tokens can be ``register``-ed under the hash of its token prefix; a later request
    with the same prefix ``take``-s it instead of recomputing it (reference count +1).
    A page whose count drops to 0 stays cached but allocatable: uncached free pages are
    handed out first (a plain stack, sliced: the per-step decode path allocates and frees
    hundreds of pages), cached ones after them in least-recently-freed order (evicted).
    """

    def __init__(self, num_blocks: int, available: int | None = None):
        if num_blocks < 2:
            raise ValueError("need at least 2 KV blocks")
        self.num_blocks = num_blocks
        self.available = num_blocks if available is None else max(2, min(available, num_blocks))
        self._ref = [0] * num_blocks        # plain lists: per-page Python ops beat numpy's per-call
        self._hashed = bytearray(num_blocks)  # overhead at the few pages a step touches
        self._free = list(range(self.available - 1, 0, -1))  # uncached free pages; pop() yields 1, 2, ...
        self._cached_free: collections.OrderedDict[int, None] = collections.OrderedDict()  # LRU first
        self._hash_of: dict[int, int] = {}
        self._by_hash: dict[int, int] = {}

    def grow(self, available: int) -> int:
        """Make page ids [self.available, available) allocatable; returns how many were added."""
        available = min(available, self.num_blocks)
        if available <= self.available:
            return 0
        self._free[:0] = range(available - 1, self.available - 1, -1)  # below the older free ids
        added = available - self.available
        self.available = available
        return added

    @property
    def num_free(self) -> int:
        return len(self._free) + len(self._cached_free)

    @property
    def num_cached(self) -> int:
        return len(self._by_hash)

    def can_allocate(self, n: int) -> bool:
        return n <= self.num_free

    def allocate(self, n: int) -> list[int]:
        if n > self.num_free:
            raise MemoryError(f"KV cache exhausted: want {n}, free {self.num_free}")
        k = min(n, len(self._free))
        out = self._free[-k:][::-1] if k else []
        del self._free[len(self._free) - k:]
        for _ in range(n - k):  # evict least recently freed cached pages
            b, _ = self._cached_free.popitem(last=False)
            del self._by_hash[self._hash_of.pop(b)]
            self._hashed[b] = 0
            out.append(b)
        ref = self._ref
        for b in out:
            ref[b] = 1
        return out

    def free(self, blocks) -> None:
        ref, hashed, plain = self._ref, self._hashed, []
        for b in reversed(blocks):  # a sequence holds each of its pages once
            r = ref[b] - 1
            ref[b] = r
            if r == 0:
                if hashed[b]:
                    self._cached_free[b] = None
                else:
                    plain.append(b)
        self._free.extend(plain)

    # ----------------------------------------------------------- prefix cache --
    def lookup(self, h: int) -> int | None:
        return self._by_hash.get(h)

    def take(self, b: int) -> None:
        """One more reference to cached page ``b`` (a prefix hit)."""
        if self._ref[b] == 0:
            del self._cached_free[b]
        self._ref[b] += 1

    def register(self, b: int, h: int) -> None:
        """Page ``b`` (held, count >= 1) now holds the computed full page of prefix hash ``h``."""
        if h not in self._by_hash and not self._hashed[b]:
            self._by_hash[h] = b
            self._hash_of[b] = h
            self._hashed[b] = 1

    def usage(self) -> float:
        return 1.0 - self.num_free / (self.available - 1)


def prefix_hashes(tokens, n_blocks: int, start: int = 0, prev: bytes = b"") -> list[bytes]:
    """Chained digests of full pages [start, n_blocks) of ``tokens``: page i's key is
    BLAKE2b-128(key of page i-1 || token ids of page i as int64), so equal keys mean equal
    prefixes.  A cryptographic digest, not Python's ``hash()`` (int hashes are the value mod
    2^61 - 1 and tuple hashing is not collision resistant): a crafted prompt must not be able
    to collide with another tenant's prefix and be served its KV pages (the flaw behind
    vLLM's CVE-2025-25183)."""
    import hashlib

    import numpy as np

    out = []
    h = prev
    arr = np.asarray(tokens[start * BLOCK_SIZE:n_blocks * BLOCK_SIZE], dtype=np.int64)
    for j, i in enumerate(range(start, n_blocks)):
        h = hashlib.blake2b(h + arr[j * BLOCK_SIZE:(j + 1) * BLOCK_SIZE].tobytes(), digest_size=16).digest()
        out.append(h)
    return out


def blocks_needed(num_tokens: int) -> int:
    return (num_tokens + BLOCK_SIZE - 1) // BLOCK_SIZE
