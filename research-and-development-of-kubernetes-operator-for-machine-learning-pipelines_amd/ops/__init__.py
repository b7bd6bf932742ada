"""Hand-written gfx950 HIP kernels, exposed as ``torch.ops.mlop.*``.

``load()`` loads the in-tree ``_C.so`` (built by ``mlopamd.ops.build``).  On a
GPU process the extension is REQUIRED: every public function here raises if it
is missing instead of silently running a PyTorch fallback.  CPU tensors (unit
tests of the scheduler / engine logic in a GPU-less container) are routed to
``mlopamd.ops.reference`` — the plain fp32 PyTorch definitions that the GPU
numerics tests also use as their oracle.
"""
from __future__ import annotations

import math
import os
from pathlib import Path

import torch

from . import reference as ref

_LIB = Path(__file__).resolve().parent / "_C.so"
_loaded = False


class StaleExtension(RuntimeError):
    pass


def load(build_if_missing: bool = True) -> bool:
    """Load the in-tree extension; build it first if it is missing and hipcc exists.
    The library carries the sha256 of the sources it was compiled from
    (``torch.ops.mlop.src_hash``): a binary that does not match this tree's sources is
    refused (``StaleExtension``), never run (a kernel replaces the
    torch op once it passes; the tested ``.so`` must be the one the sources describe)."""
    global _loaded
    if _loaded:
        return True
    from .build import source_hash

    want = source_hash()
    if not _LIB.exists() and build_if_missing:
        from .build import build

        build()
    torch.ops.load_library(str(_LIB))
    got = torch.ops.mlop.src_hash()
    if got != want:
        raise StaleExtension(f"{_LIB} was built from sources {got}, this tree is {want}: "
                             "rebuild with `python -m mlopamd.ops.build`")
    _loaded = True
    load_gemm_table()
    return True


def available() -> bool:
    try:
        return load(build_if_missing=False)
    except Exception:  # noqa: BLE001
        return False


def _need_gpu():
    if not _loaded:
        load()


_SK_READY: set = set()


def _sk_reserve(dev) -> None:
    """Stream-K tail buffers of the ping-pong GEMM (128 MB partials + counters) on this
    device: allocated once, on the first eager GEMM (never inside a graph capture; until
    they exist the kernel runs its plain data-parallel grid)."""
    i = dev.index if dev.index is not None else torch.cuda.current_device()
    if i in _SK_READY or torch.cuda.is_current_stream_capturing():
        return
    with torch.cuda.device(i):
        torch.ops.mlop.gemm_sk_reserve()
    _SK_READY.add(i)


def library_path() -> str:
    return str(_LIB)


# ---------------------------------------------------------------- wrappers --

def rmsnorm(x: torch.Tensor, w: torch.Tensor, eps: float, out: torch.Tensor | None = None):
    if not x.is_cuda:
        return ref.rmsnorm(x, w, eps)
    _need_gpu()
    out = torch.empty_like(x) if out is None else out
    torch.ops.mlop.rmsnorm(out, x, w, eps)
    return out


def add_rmsnorm(x: torch.Tensor, residual: torch.Tensor, w: torch.Tensor, eps: float,
                out: torch.Tensor | None = None):
    """residual <- residual + x (bf16); returns rmsnorm(residual) * w."""
    if not x.is_cuda:
        y, r = ref.add_rmsnorm(x, residual, w, eps)
        residual.copy_(r)
        if out is not None:
            out.copy_(y)
            return out
        return y
    _need_gpu()
    out = torch.empty_like(x) if out is None else out
    torch.ops.mlop.add_rmsnorm(out, residual, x, w, eps)
    return out


def rope_cache(qkv, positions, cos_sin, slots, k_cache, v_cache, n_q_heads: int,
               q_out: torch.Tensor | None = None):
    T = qkv.shape[0]
    D = k_cache.shape[3]
    if not qkv.is_cuda:
        q = ref.rope_cache(qkv, positions, cos_sin, slots, k_cache, v_cache, n_q_heads)
        if q_out is not None:
            q_out.copy_(q)
            return q_out
        return q
    _need_gpu()
    q_out = torch.empty(T, n_q_heads, D, dtype=qkv.dtype, device=qkv.device) if q_out is None else q_out
    torch.ops.mlop.rope_cache(q_out, k_cache, v_cache, qkv, positions, cos_sin, slots)
    return q_out


def silu_mul(x: torch.Tensor, out: torch.Tensor | None = None):
    if not x.is_cuda:
        return ref.silu_mul(x)
    _need_gpu()
    I = x.shape[-1] // 2
    out = torch.empty(*x.shape[:-1], I, dtype=x.dtype, device=x.device) if out is None else out
    torch.ops.mlop.silu_mul(out, x)
    return out


def embedding(ids: torch.Tensor, table: torch.Tensor, vocab_start: int = 0,
              out: torch.Tensor | None = None):
    if not ids.is_cuda:
        return ref.embedding(ids, table, vocab_start)
    _need_gpu()
    out = torch.empty(ids.numel(), table.shape[1], dtype=table.dtype, device=table.device) if out is None else out
    torch.ops.mlop.embedding(out, table, ids, vocab_start)
    return out


_NO_SEM: dict = {}


def _no_sem(device):
    t = _NO_SEM.get(device)
    if t is None:
        t = _NO_SEM[device] = torch.empty(0, dtype=torch.int32, device=device)
    return t


def paged_attention(q, k_cache, v_cache, meta, out: torch.Tensor | None = None):
    """Ragged paged attention; ``meta`` is a ``mlopamd.runtime.attn_meta.AttnMeta``.
    Decode / short rows run on the 16-q-row tiles (``tile_*``), prompt chunks on
    the flash-prefill tiles (``ptile_*``); both write disjoint rows of ``out``."""
    if not q.is_cuda:
        return ref.paged_attention(q, k_cache, v_cache, meta)
    _need_gpu()
    out = torch.empty_like(q) if out is None else out
    scale = 1.0 / math.sqrt(q.shape[-1])
    if meta.tile_seq.numel():
        sem = getattr(meta, "part_sem", None)
        if sem is None:
            sem = _no_sem(q.device)
        torch.ops.mlop.paged_attention(out, meta.part_o, meta.part_ml, sem, q, k_cache, v_cache,
                                       meta.block_tables, meta.tile_seq, meta.tile_q0, meta.q_start,
                                       meta.q_len, meta.ctx_len, scale, meta.part_tokens, meta.nparts)
    pts = getattr(meta, "ptile_seq", None)
    if pts is not None and pts.numel():
        # prompt chunks: K7 flash prefill (128 q-rows per workgroup, K/V via LDS-DMA)
        torch.ops.mlop.flash_prefill(out, q, k_cache, v_cache, meta.block_tables, pts, meta.ptile_q0,
                                     meta.q_start, meta.q_len, meta.ctx_len, scale)
    return out


EPI_NONE, EPI_SILU_MUL = 0, 1


def gemm(x: torch.Tensor, w: torch.Tensor, out: torch.Tensor | None = None, epi: int = EPI_NONE):
    """y = epi(x @ w^T), w [N, K] bf16.  EPI_SILU_MUL expects gate/up rows
    interleaved in groups of 16 (``interleave_gate_up``) and returns N/2 columns."""
    N = w.shape[0]
    out_n = N if epi == EPI_NONE else N // 2
    if not x.is_cuda:
        y = torch.nn.functional.linear(x, w) if x.dtype != torch.bfloat16 else \
            torch.nn.functional.linear(x.float(), w.float()).to(x.dtype)
        if epi == EPI_SILU_MUL:
            y = ref.silu_mul(deinterleave_cols(y))
        if out is not None:
            out.copy_(y.view_as(out))
            return out
        return y
    _need_gpu()
    lead = x.shape[:-1]
    x2 = x.reshape(-1, x.shape[-1])
    if x2.stride(-1) != 1 or x2.stride(0) % 8:
        x2 = x2.contiguous()
    M, K = x2.shape
    o2 = torch.empty(M, out_n, dtype=x.dtype, device=x.device) if out is None else out.view(M, out_n)
    _GEMM_IMPL[_gemm_backend(M, N, K, epi, x2, w, o2)](x2, w, o2, epi)
    return o2.view(*lead, out_n) if out is None else out


def _gemm_mlop(x2, w, o2, epi):
    _sk_reserve(x2.device)
    M, K = x2.shape
    nws = torch.ops.mlop.gemm_workspace(M, w.shape[0], K, epi)
    ws = torch.empty(max(nws, 1), dtype=torch.float32, device=x2.device) if nws else _EMPTY.get(x2.device)
    torch.ops.mlop.gemm(o2, x2, w, ws, epi)


def _gemm_hipblaslt(x2, w, o2, epi):
    """Plain library GEMM (hipBLASLt via torch.matmul); the SiLU-mul epilogue
    then runs as the separate interleaved silu_mul kernel."""
    if epi == EPI_NONE:
        torch.matmul(x2, w.t(), out=o2)
    else:
        torch.ops.mlop.silu_mul(o2, torch.matmul(x2, w.t()), 1)


_GEMM_IMPL = {"mlop": _gemm_mlop, "hipblaslt": _gemm_hipblaslt}
_GEMM_CHOICE: dict = {}
# Which GEMM runs a projection: "mlop" (default) = the hand-written kernels (GEMV / MFMA tiles /
# ping-pong 256x256 with fused epilogues) wherever their tiling contract holds; "auto" = the
# per-shape timed choice against hipBLASLt (+ its separate epilogue op), seeded from the shipped
# table -- kept as the A/B reference (profiles/r03_gemm_fourwave.md: equal end to end since the
# two-phase ping-pong loop); "hipblaslt" = library only.
GEMM_BACKEND_DEFAULT = "mlop"
GEMM_BACKEND = os.environ.get("MLOP_GEMM_BACKEND", GEMM_BACKEND_DEFAULT)  # mlop | auto | hipblaslt
_GEMM_USED: dict = {}  # (M bucket, N, K, epi) -> backend that actually ran (gemm_used())


def gemm_used() -> dict:
    """{backend: number of distinct projection shapes it ran} since the last reset."""
    out = {"mlop": 0, "hipblaslt": 0}
    for c in _GEMM_USED.values():
        out[c] = out.get(c, 0) + 1
    return out


def reset_gemm_used() -> None:
    _GEMM_USED.clear()


def _mbucket(M: int) -> int:
    """Autotune key for the row count: powers of two up to 256 (GEMV / narrow-tile
    regimes), then every 256 rows: above one tile row the winner flips with how the
    256-row tiles fill the 256 CUs (e.g. QKV at M=2040 is 192 tiles = 3/4 of the chip
    for the fused RoPE kernel, while hipBLASLt's stream-K does not care), so
    power-of-two buckets let the first M seen in [1025, 2048] decide for all of them."""
    if M > 256:
        return (M + 255) // 256 * 256
    b = 1
    while b < M:
        b <<= 1
    return b


_FLUSH: dict = {}
COLD_TUNE_MAX_M = 64  # at or below this M a projection streams its weights once per step


def _flush_caches(dev) -> None:
    """Evict L2 and the 256 MB Infinity Cache (MALL) by writing 512 MB: a decode
    step reads each weight once, cold, so hot-cache timings flatter whichever
    kernel re-reads better from MALL (the gate_up GEMV vs hipBLASLt flips)."""
    buf = _FLUSH.get(dev)
    if buf is None:
        buf = _FLUSH[dev] = torch.empty(512 << 20, dtype=torch.uint8, device=dev)
    buf.fill_(1)


def _time_candidates(cands, M: int, dev, reps: int = 5, rounds: int = 3) -> dict:
    """ms per call per candidate: cold caches before every rep when M is decode-sized;
    otherwise the best of ``rounds`` interleaved rounds of ``reps`` back-to-back calls
    (one 3-call sample per candidate mis-picked QKV at M=2048 by 20-30%: clocks and
    heuristic warm-up drift between the two candidates' samples)."""
    cold = M <= COLD_TUNE_MAX_M
    times = {name: float("inf") for name, _ in cands}
    for name, fn in cands:
        fn()  # warm (kernel selection, lazy init)
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(1 if cold else rounds):
        for name, fn in cands:
            tot = 0.0
            if cold:
                for _ in range(reps):
                    _flush_caches(dev)
                    s.record()
                    fn()
                    e.record()
                    e.synchronize()
                    tot += s.elapsed_time(e)
            else:
                s.record()
                for _ in range(reps):
                    fn()
                e.record()
                e.synchronize()
                tot = s.elapsed_time(e)
            times[name] = min(times[name], tot / reps)
    return times


def _gemm_backend(M, N, K, epi, x2, w, o2) -> str:
    c = _gemm_backend_choice(M, N, K, epi, x2, w, o2)
    _GEMM_USED[(_mbucket(M), N, K, epi)] = c
    return c


def _gemm_backend_choice(M, N, K, epi, x2, w, o2) -> str:
    """Per-shape choice between the hand-written MFMA kernel and hipBLASLt: the configured
    backend, or (``auto``) measured once per (M bucket, N, K, epilogue) on first eager use
    (never during graph capture).  ``gemm_choices()`` reports the table."""
    if N % 8 or K % 64 or (epi != EPI_NONE and N % 32):
        return "hipblaslt"  # shapes outside the MFMA kernel's tiling contract (e.g. tiny routers)
    if GEMM_BACKEND != "auto":
        return GEMM_BACKEND
    key = (_mbucket(M), N, K, epi)
    c = _GEMM_CHOICE.get(key)
    if c is not None:
        return c
    if AUTOTUNE_FROZEN:
        return _nearest_choice(key) or "mlop"
    if torch.cuda.is_current_stream_capturing():
        return "mlop"
    times = _time_candidates([(n, (lambda f=f: f(x2, w, o2, epi))) for n, f in _GEMM_IMPL.items()], M, x2.device)
    c = min(times, key=times.get)
    _GEMM_CHOICE[key] = c
    _GEMM_TIMES[key] = times
    return c


_GEMM_TIMES: dict = {}
EPI_ADD_RMSNORM = 2  # autotune key only
# Frozen: a key never timed takes the choice of the nearest timed row count of the same
# (N, K, epilogue) instead of timing both candidates on the spot (a serving loop, or a
# benchmark's timed steps, must not stall on a first-seen batch size).  freeze_autotune().
AUTOTUNE_FROZEN = False


def freeze_autotune(frozen: bool = True) -> None:
    global AUTOTUNE_FROZEN
    AUTOTUNE_FROZEN = frozen


def _nearest_choice(key):
    mb, N, K, epi = key
    best = None
    for (m2, n2, k2, e2), c in _GEMM_CHOICE.items():
        if (n2, k2, e2) == (N, K, epi):
            d = abs(m2 - mb)
            if best is None or d < best[0]:
                best = (d, c)
    return best[1] if best else None


def gemm_add_rmsnorm(x, w, residual, norm_w, eps: float):
    """Decoder projection + residual + norm: residual <- residual + x @ w^T (bf16);
    returns rmsnorm(residual) * norm_w.  On GPU the split-K MFMA GEMM's reduce
    pass does the add and the norm (one launch fewer, one activation round trip
    fewer) when that beats hipBLASLt + add_rmsnorm for the shape."""
    if not x.is_cuda:
        return add_rmsnorm(gemm(x, w), residual, norm_w, eps)
    _need_gpu()
    x2 = x.reshape(-1, x.shape[-1])
    if x2.stride(-1) != 1 or x2.stride(0) % 8:
        x2 = x2.contiguous()
    M, K = x2.shape
    N = w.shape[0]
    _sk_reserve(x.device)  # the GEMV epilogue form's grid ticket lives in the stream-K scratch
    # decode sizes (M <= 4): the GEMV with the add + RMSNorm as its epilogue (grid ticket, one
    # launch); larger M: the split-K reduce pass does them
    nws = torch.ops.mlop.gemm_workspace(M, N, K, EPI_ADD_RMSNORM) if (K % 8 == 0 and N % 8 == 0) else 0

    def fused(res):
        ws = torch.empty(nws, dtype=torch.float32, device=x.device)
        out = torch.empty(M, N, dtype=x.dtype, device=x.device)
        if not torch.ops.mlop.gemm_add_rmsnorm(out, res, x2, w, norm_w, ws, eps):
            raise RuntimeError("fused path not applicable")
        return out

    def unfused(res):
        return add_rmsnorm(gemm(x2, w), res, norm_w, eps)

    key = (_mbucket(M), N, K, EPI_ADD_RMSNORM)
    if nws == 0 or GEMM_BACKEND == "hipblaslt":
        return unfused(residual)  # the GEMM inside records its own backend
    if GEMM_BACKEND == "mlop":
        _GEMM_USED[key] = "mlop"
        return fused(residual)
    c = _GEMM_CHOICE.get(key)
    if c is None and AUTOTUNE_FROZEN:
        c = _nearest_choice(key)
    if c is None and not torch.cuda.is_current_stream_capturing():
        scratch = residual.clone()
        times = _time_candidates([("mlop", lambda: fused(scratch)), ("hipblaslt", lambda: unfused(scratch))],
                                 M, x.device)
        c = min(times, key=times.get)
        _GEMM_CHOICE[key], _GEMM_TIMES[key] = c, times
    if c in (None, "mlop"):
        _GEMM_USED[key] = "mlop"
        return fused(residual)
    return unfused(residual)


EPI_ROPE = 3  # QKV projection + RoPE + paged-cache stores in the GEMM epilogue


def qkv_rope_cache(x, w, positions, cos_sin, slots, k_cache, v_cache, n_q_heads: int,
                   q_out: torch.Tensor | None = None):
    """q_out <- RoPE(x @ Wq^T); k_cache / v_cache[slot] <- RoPE(x @ Wk^T), x @ Wv^T.

    On GPU the MFMA GEMM does the rotation and the cache scatter from its LDS-staged
    C tile (one launch, no [T, (Hq+2Hkv)D] round trip through HBM) when the M of the
    step takes whole-head tiles (M > 256); the per-shape choice against hipBLASLt +
    rope_cache is timed like every other projection (key epi = EPI_ROPE)."""
    T = x.shape[0]
    D = k_cache.shape[3]
    if not x.is_cuda:
        return rope_cache(gemm(x, w), positions, cos_sin, slots, k_cache, v_cache, n_q_heads, q_out)
    _need_gpu()
    x2 = x if (x.stride(-1) == 1 and x.stride(0) % 8 == 0) else x.contiguous()
    M, K = x2.shape
    N = w.shape[0]
    q_out = torch.empty(T, n_q_heads, D, dtype=x.dtype, device=x.device) if q_out is None else q_out

    _sk_reserve(x.device)

    def fused():
        if not torch.ops.mlop.gemm_rope_cache(q_out, k_cache, v_cache, x2, w, positions, cos_sin, slots):
            raise RuntimeError("fused QKV+RoPE tiling not applicable")
        return q_out

    def unfused():
        return rope_cache(gemm(x2, w), positions, cos_sin, slots, k_cache, v_cache, n_q_heads, q_out)

    key = (_mbucket(M), N, K, EPI_ROPE)
    if GEMM_BACKEND == "hipblaslt" or not torch.ops.mlop.gemm_rope_supported(M, N, K):
        return unfused()
    if GEMM_BACKEND == "mlop":
        _GEMM_USED[key] = "mlop"
        return fused()
    c = _GEMM_CHOICE.get(key)
    if c is None and AUTOTUNE_FROZEN:
        c = _nearest_choice(key)
    if c is None and not torch.cuda.is_current_stream_capturing():
        # fused() re-writes the same cache slots with the same values: idempotent
        times = _time_candidates([("mlop", fused), ("hipblaslt", unfused)], M, x.device)
        c = min(times, key=times.get)
        _GEMM_CHOICE[key], _GEMM_TIMES[key] = c, times
    if c in (None, "mlop"):
        _GEMM_USED[key] = "mlop"
        return fused()
    return unfused()


# ---- norm chain (large-M TP=1 decoder): the add + RMSNorm passes folded into the GEMMs ----
# O / down run C = residual += x @ w^T and leave the new residual's per-row sums of squares in
# an ss buffer (ss_buffer: [M, N / 128] partials, one per 128 columns, written not accumulated,
# then the [M] row totals, summed in a fixed order by the last tile of each row band:
# deterministic); gate_up / QKV read the un-normalised residual and scale each accumulator row
# by rsqrt(total / K + eps) =
# RMSNorm after the GEMM, with the norm weight folded into their weights (LlamaModel.fold_norms).
# "1" (default): on where every GEMM of the chain runs on the four-wave kernel; "0" off;
# "force": also on CPU / any shape through the torch reference below (plumbing tests set it).
NORM_CHAIN = "1"


# The decode (M <= 4) form of the chain runs on the GEMV (gemv.hip EPI_RES / PRO_RS): O and down
# add into the residual in place, QKV and gate_up take each row's factor from the residual
# chunks they stream, so a layer has no add + RMSNorm launch.  False keeps the decode norms (the
# GPU tests' A/B).
GEMV_CHAIN = True
GEMV_CHAIN_MAX_M = 4  # = gemv.hip gemv_chain_max_m (the GEMV form; the torch reference's decode form)


def decode_chain_max_m() -> int:
    """Rows the decode form of the norm chain takes: the GEMV up to 4 rows, then the
    weight-streaming MFMA kernel (gemm_ws.hip) up to ``gemm_ws_max_m`` (64; the
    ``gemm_ws_max_m`` op is its A/B switch).  Without the extension (CPU): the GEMV bound."""
    if _loaded:
        return int(torch.ops.mlop.decode_chain_max_m())
    return GEMV_CHAIN_MAX_M


def norm_chain_ok(M: int, H: int, shapes, device=None, epis=None) -> bool:
    """True when the chain can run at M rows: hidden size H (ss groups of 128 columns, 16 per
    quad of lanes) and every (N, K) GEMM of the chain on the four-wave kernel, with the band
    tickets' scratch reserved on ``device`` and one ticket per 256-row band (w4_chain_ok checks
    everything launch_w4_chain does, so the chain is decided once per forward and never refused
    after a residual was updated in place).  At M <= 4 every GEMM must take the GEMV form
    instead (``epis``: each shape's epilogue, default plain)."""
    if NORM_CHAIN == "force":
        return H % 128 == 0
    if NORM_CHAIN == "0" or GEMM_BACKEND != "mlop" or H % 256:
        return False
    if device is not None and torch.device(device).type != "cuda":
        return False  # the torch reference path (CPU) has no chain kernels
    _need_gpu()
    if M <= decode_chain_max_m():
        epis = epis or [EPI_NONE] * len(shapes)
        return GEMV_CHAIN and all(bool(torch.ops.mlop.gemv_chain_supported(M, N, K, e))
                                  for (N, K), e in zip(shapes, epis))
    if device is not None and torch.device(device).type == "cuda":
        _sk_reserve(torch.device(device))
    if M <= 64 and epis is not None:
        # 5-64 rows: the planner's small tiles (O / down finish their split-K and leave the row
        # sums of squares, gate_up / QKV scale their rows: gemm.hip mid_chain_ok)
        return all(bool(torch.ops.mlop.mid_chain_ok(M, N, K, e)) for (N, K), e in zip(shapes, epis))
    return all(bool(torch.ops.mlop.w4_chain_ok(M, N, K)) for N, K in shapes)


def ss_buffer(M: int, H: int, device) -> torch.Tensor:
    """fp32 [M * (H / 128 + 1)]: the [M, H / 128] partials, then the [M] row totals."""
    return torch.empty(M * (H // 128 + 1), dtype=torch.float32, device=device)


def ss_init(x: torch.Tensor, ss: torch.Tensor) -> torch.Tensor:
    """ss (ss_buffer) <- x's row partials and totals where the torch reference of the chain
    will read them; the GPU chain's decode (GEMV) form takes its row factors from x itself."""
    if x.is_cuda and NORM_CHAIN != "force":
        return ss
    M, H = x.shape
    part, tot = ss_parts(ss, M, H)
    part.copy_(x.float().pow(2).view(M, H // 128, 128).sum(-1))
    tot.copy_(part.sum(-1))
    return ss


def ss_parts(ss: torch.Tensor, M: int, H: int):
    """(partials [M, H / 128], totals [M]) views of an ss_buffer."""
    G = H // 128
    return ss[:M * G].view(M, G), ss[M * G:M * (G + 1)]


def _rinv_ref(ss: torch.Tensor, M: int, K: int, eps: float) -> torch.Tensor:
    return torch.rsqrt(ss_parts(ss, M, K)[1].view(M, 1) / K + eps)


def gemm_res_ss(x, w, residual, ss_out):
    """residual [M, N] += x @ w^T in place (bf16); ss_out (ss_buffer(M, N)) <- the new residual
    rows' partial sums of squares and totals.  The four-wave kernel's W4_ADD_SS epilogue on GPU."""
    if x.is_cuda and NORM_CHAIN != "force":
        _need_gpu()
        _sk_reserve(x.device)
        if not torch.ops.mlop.gemm_res_ss(residual, x, w, ss_out):
            raise RuntimeError("norm chain: shape not on the four-wave kernel")
        _GEMM_USED[(_mbucket(x.shape[0]), w.shape[0], w.shape[1], EPI_ADD_SS)] = "mlop"
        return residual
    residual.copy_((residual.float() + x.float() @ w.float().t()).to(residual.dtype))
    M, N = residual.shape
    part, tot = ss_parts(ss_out, M, N)
    part.copy_(residual.float().pow(2).view(M, N // 128, 128).sum(-1))
    tot.copy_(part.sum(-1))
    return residual


def gemm_rs(x, w, ss, eps: float, epi: int = EPI_NONE):
    """epi(rmsnorm_unit(x) @ w^T) with the row factors from ss (gemm_res_ss's partials): the
    normalisation is applied to the accumulators (W4_RS), x is the raw residual."""
    M, K = x.shape
    N = w.shape[0]
    if x.is_cuda and NORM_CHAIN != "force":
        _need_gpu()
        _sk_reserve(x.device)
        out = torch.empty(M, N if epi == EPI_NONE else N // 2, dtype=x.dtype, device=x.device)
        if not torch.ops.mlop.gemm_rs(out, x, w, ss, eps, epi):
            raise RuntimeError("norm chain: shape not on the four-wave kernel")
        _GEMM_USED[(_mbucket(M), N, K, epi | EPI_RS)] = "mlop"
        return out
    return gemm((x.float() * _rinv_ref(ss, M, K, eps)).to(x.dtype), w, epi=epi)


def qkv_rope_cache_rs(x, w, positions, cos_sin, slots, k_cache, v_cache, n_q_heads: int, ss, eps: float):
    """qkv_rope_cache of rmsnorm_unit(x) with the row factors from ss (norm chain)."""
    M, K = x.shape
    if x.is_cuda and NORM_CHAIN != "force":
        _need_gpu()
        _sk_reserve(x.device)
        q_out = torch.empty(M, n_q_heads, k_cache.shape[3], dtype=x.dtype, device=x.device)
        if not torch.ops.mlop.gemm_rs_rope(q_out, k_cache, v_cache, x, w, positions, cos_sin, slots, ss, eps):
            raise RuntimeError("norm chain: shape not on the four-wave kernel")
        _GEMM_USED[(_mbucket(M), w.shape[0], K, EPI_ROPE | EPI_RS)] = "mlop"
        return q_out
    return rope_cache(gemm((x.float() * _rinv_ref(ss, M, K, eps)).to(x.dtype), w), positions, cos_sin, slots, k_cache,
                      v_cache, n_q_heads)


EPI_ADD_SS, EPI_RS = 4, 8  # norm-chain epilogue flags (gemm_used() keys; gemm_w4.hip W4_ADD_SS / W4_RS)


GEMM_TABLE = Path(os.environ.get("MLOP_GEMM_TABLE", str(Path(__file__).with_name("gemm_table_gfx950.json"))))


def load_gemm_table(path: str | os.PathLike | None = None) -> int:
    """Seed the per-shape backend choice from a table measured earlier on this
    architecture (a tuning database, like hipBLASLt's own): a predictor then skips
    re-timing every projection shape during start-up / graph capture.  Shapes not
    in the table are still timed on first use.  Returns the number of entries."""
    p = Path(path) if path else GEMM_TABLE
    if os.environ.get("MLOP_GEMM_TABLE") == "off" or not p.exists():
        return 0
    import json

    d = json.loads(p.read_text())
    n = 0
    for mb, N, K, epi, choice in d.get("entries", []):
        if choice in _GEMM_IMPL:
            _GEMM_CHOICE.setdefault((int(mb), int(N), int(K), int(epi)), choice)
            n += 1
    return n


def save_gemm_table(path: str | os.PathLike | None = None) -> str:
    """Write the choices measured so far, merged over the shipped table and over an
    existing file at ``path`` (so a table saved elsewhere is a complete drop-in)."""
    import json

    p = Path(path) if path else GEMM_TABLE
    entries = {}
    for src in dict.fromkeys([GEMM_TABLE, p]):
        if src.exists():
            for e in json.loads(src.read_text()).get("entries", []):
                entries[tuple(e[:4])] = e[4]
    for k, c in _GEMM_CHOICE.items():
        if k in _GEMM_TIMES:  # only shapes actually timed in this process
            entries[k] = c
    rows = [json.dumps([*k, c]) for k, c in sorted(entries.items())]
    p.write_text('{"arch": "gfx950", "entries": [\n' + ",\n".join(rows) + "\n]}\n")
    return str(p)


def gemm_choices() -> list:
    return [dict(M_bucket=k[0], N=k[1], K=k[2], epi=k[3], choice=_GEMM_CHOICE[k],
                 **{f"{n}_us": round(t * 1e3, 1) for n, t in _GEMM_TIMES.get(k, {}).items()})
            for k in sorted(_GEMM_CHOICE)]


class _EmptyCache(dict):
    def get(self, dev):  # noqa: D401
        if dev not in self:
            self[dev] = torch.empty(0, dtype=torch.float32, device=dev)
        return self[dev]


_EMPTY = _EmptyCache()


def interleave_gate_up(gate: torch.Tensor, up: torch.Tensor, group: int = 16) -> torch.Tensor:
    """[I, K] gate and up -> [2I, K] rows [g0..g15, u0..u15, g16.., u16.., ...] (EPI_SILU_MUL layout)."""
    I, K = gate.shape
    assert I % group == 0
    return torch.stack([gate.view(I // group, group, K), up.view(I // group, group, K)], 1).reshape(2 * I, K)


def deinterleave_rows(w: torch.Tensor, group: int = 16) -> torch.Tensor:
    """Inverse of interleave_gate_up: [2I, K] interleaved -> [2I, K] = [gate; up]."""
    n2, K = w.shape
    v = w.view(n2 // (2 * group), 2, group, K)
    return torch.cat([v[:, 0].reshape(-1, K), v[:, 1].reshape(-1, K)], 0)


def deinterleave_cols(y: torch.Tensor, group: int = 16) -> torch.Tensor:
    """Columns of x @ W_interleaved^T -> [gate | up] column order."""
    *lead, n2 = y.shape
    v = y.reshape(-1, n2 // (2 * group), 2, group)
    return torch.cat([v[:, :, 0].reshape(-1, n2 // 2), v[:, :, 1].reshape(-1, n2 // 2)], -1).view(*lead, n2)


def argmax(logits: torch.Tensor) -> torch.Tensor:
    if not logits.is_cuda:
        return logits.argmax(-1)
    _need_gpu()
    out = torch.empty(logits.shape[0], dtype=torch.int64, device=logits.device)
    torch.ops.mlop.argmax(out, logits)
    return out


SAMPLE_MAX_CAND = 1024  # sampling.hip kMaxCand: top_k above this (or 0) draws from the whole row


def sample(logits, temps, top_ks, top_ps, uniform, full: bool | None = None) -> torch.Tensor:
    """temperature / top-k / top-p draw per row (K10).  ``full``: whether any non-greedy row has
    top_k = 0 or > SAMPLE_MAX_CAND (those rows are drawn from the whole vocabulary); None =
    find out from ``top_ks`` / ``temps`` (one device sync)."""
    if not logits.is_cuda:
        from ..runtime.sampler import sample_reference

        return sample_reference(logits, temps, top_ks, top_ps, uniform)
    _need_gpu()
    if full is None:
        full = bool((((top_ks <= 0) | (top_ks > SAMPLE_MAX_CAND)) & (temps > 0)).any())
    out = torch.empty(logits.shape[0], dtype=torch.int64, device=logits.device)
    torch.ops.mlop.sample(out, logits, temps, top_ks, top_ps, uniform, bool(full))
    return out


__all__ = ["argmax", "sample", "load","available", "library_path", "rmsnorm", "add_rmsnorm", "rope_cache",
           "silu_mul", "embedding", "paged_attention", "ref"]


# ------------------------------------------------------------------ MoE --
# Static-shape MoE primitives (graph-capturable): the permuted batch keeps
# T*k rows; offsets[n_local] is the number of valid rows.

def moe_route(logits: torch.Tensor, top_k: int):
    """softmax -> top-k -> renormalise; logits bf16 [T, E] -> (w f32 [T,k], idx int32 [T,k])."""
    if not logits.is_cuda:
        return ref.moe_route(logits, top_k)
    _need_gpu()
    T = logits.shape[0]
    w = torch.empty(T, top_k, dtype=torch.float32, device=logits.device)
    idx = torch.empty(T, top_k, dtype=torch.int32, device=logits.device)
    torch.ops.mlop.moe_route(w, idx, logits.contiguous())
    return w, idx


def moe_permute(x, topi, e0: int, n_local: int):
    """Group routed slots by local expert.  Returns (xp [T*k, H], offsets [n_local+1],
    src [T*k] row->slot, inv [T*k] slot->row or -1)."""
    if not x.is_cuda:
        return ref.moe_permute(x, topi, e0, n_local)
    _need_gpu()
    T, k = topi.shape
    dev = x.device
    xp = torch.empty(T * k, x.shape[1], dtype=x.dtype, device=dev)
    offsets = torch.empty(n_local + 1, dtype=torch.int32, device=dev)
    src = torch.empty(T * k, dtype=torch.int32, device=dev)
    inv = torch.empty(T * k, dtype=torch.int32, device=dev)
    torch.ops.mlop.moe_permute(xp, offsets, src, inv, x.contiguous(), topi.contiguous(), e0, n_local)
    return xp, offsets, src, inv


def moe_dispatch_small(x, router_w, top_k: int, e0: int, n_local: int, pro=None):
    """Decode-size MoE dispatch in ONE launch (router GEMV + route + sort + gather, moe.hip):
    returns (topw, topi, xp, offsets, src, inv) or None when the shape is not on this path
    (more than 16 tokens, CPU tensors).  ``pro=(y, residual, norm_w, eps)``: x is not given
    (pass y); the launch first does residual += y, x = rmsnorm(residual) * norm_w.  On None
    nothing was written."""
    if not x.is_cuda or x.shape[0] > 16:
        return None
    _need_gpu()
    T, H = x.shape
    dev = x.device
    topw = torch.empty(T, top_k, dtype=torch.float32, device=dev)
    topi = torch.empty(T, top_k, dtype=torch.int32, device=dev)
    xp = torch.empty(T * top_k, H, dtype=x.dtype, device=dev)
    offsets = torch.empty(n_local + 1, dtype=torch.int32, device=dev)
    src = torch.empty(T * top_k, dtype=torch.int32, device=dev)
    inv = torch.empty(T * top_k, dtype=torch.int32, device=dev)
    if pro is None:
        args = (x.contiguous(), router_w, e0, n_local)
    else:  # x (= y) is only the shape carrier; the kernel writes the normed rows to xn
        y, residual, norm_w, eps = pro
        args = (torch.empty_like(y), router_w, e0, n_local, y.contiguous(), residual, norm_w, float(eps))
    if not torch.ops.mlop.moe_dispatch_small(topw, topi, xp, offsets, src, inv, *args):
        return None
    return topw, topi, xp, offsets, src, inv


def moe_dispatch_mid(x, router_w, top_k: int, e0: int, n_local: int, pro=None):
    """MoE dispatch in ONE launch (16 < T <= 16384 tokens; moe.hip): router GEMV + route
    per token workgroup, the last workgroup sorts the slots by local expert.  Returns (topw, topi,
    x, offsets, arow, inv) -- x itself (the normed rows under ``pro``) and arow [T*k], the token row
    of each permuted row: the grouped GEMM reads x through it (``grouped_gemm(a_rows=arow)``),
    there is no gathered copy -- or None when the shape is not on this path (nothing written)."""
    if not x.is_cuda or x.shape[0] <= 16:
        return None
    _need_gpu()
    T, H = x.shape
    dev = x.device
    _sk_reserve(dev)  # the launch's ticket counter lives in the stream-K scratch
    topw = torch.empty(T, top_k, dtype=torch.float32, device=dev)
    topi = torch.empty(T, top_k, dtype=torch.int32, device=dev)
    offsets = torch.empty(n_local + 1, dtype=torch.int32, device=dev)
    arow = torch.empty(T * top_k, dtype=torch.int32, device=dev)
    inv = torch.empty(T * top_k, dtype=torch.int32, device=dev)
    if pro is None:
        xs = x.contiguous()
        args = (xs, router_w.contiguous(), e0, n_local)
    else:  # the kernel writes the normed rows to xs
        y, residual, norm_w, eps = pro
        xs = torch.empty_like(y)
        args = (xs, router_w.contiguous(), e0, n_local, y.contiguous(), residual, norm_w, float(eps))
    if not torch.ops.mlop.moe_dispatch_mid(topw, topi, offsets, arow, inv, *args):
        return None
    return topw, topi, xs, offsets, arow, inv


def moe_combine_add_rmsnorm(y, inv, topw, residual, norm_w, eps: float):
    """residual <- residual + combine(y); returns rmsnorm(residual) * norm_w (one launch on GPU)."""
    if y.is_cuda:
        _need_gpu()
        out = torch.empty_like(residual)
        if torch.ops.mlop.moe_combine_add_rmsnorm(out, residual, y, inv, topw, norm_w, eps):
            return out
    return add_rmsnorm(moe_combine(y, inv, topw), residual, norm_w, eps)


def moe_down_combine_add_rmsnorm(a, w2, offsets, inv, topw, residual, norm_w, eps: float, avg_rows: int):
    """The MoE block's tail: y = grouped down GEMM of the SiLU-mul rows ``a``; residual <-
    residual + combine(y); returns rmsnorm(residual) * norm_w.  On GPU the combine sums the
    GEMM's split-K partials itself (one launch fewer than GEMM + reduce + combine)."""
    if a.is_cuda and a.shape[0] > 0:
        _need_gpu()
        _sk_reserve(a.device)
        out = torch.empty_like(residual)
        y = torch.empty(a.shape[0], w2.shape[1], dtype=a.dtype, device=a.device)
        if torch.ops.mlop.moe_down_combine_add_rmsnorm(out, residual, y, a, w2, offsets, avg_rows, inv,
                                                       topw.contiguous(), norm_w, eps):
            return out
    y = grouped_gemm(a, w2, offsets, avg_rows=avg_rows)
    return moe_combine_add_rmsnorm(y, inv, topw, residual, norm_w, eps)


def moe_combine(y, inv, topw):
    """out[t] = sum_j topw[t,j] * y[inv[t*k+j]] (inv < 0 skipped), fp32 accumulate."""
    if not y.is_cuda:
        return ref.moe_combine(y, inv, topw)
    _need_gpu()
    out = torch.empty(topw.shape[0], y.shape[1], dtype=y.dtype, device=y.device)
    torch.ops.mlop.moe_combine(out, y, inv, topw.contiguous())
    return out


def grouped_gemm(xp, w, offsets, epi: int = EPI_NONE, avg_rows: int | None = None, a_rows=None):
    """Per group e: rows offsets[e]:offsets[e+1] of xp times w[e]^T in ONE launch
    (tiles enumerate (group, m-tile) pairs on device: no host sync, graph-safe).  ``a_rows``
    [R]: permuted row r is row a_rows[r] of xp (R output rows; moe_dispatch_mid)."""
    if a_rows is not None and not xp.is_cuda:
        xp = xp[a_rows.long()]
        a_rows = None
    if not xp.is_cuda:
        y = ref.grouped_gemm(xp, w, offsets)
        return ref.silu_mul(deinterleave_cols(y)) if epi == EPI_SILU_MUL else y
    _need_gpu()
    N = w.shape[1]
    R = xp.shape[0] if a_rows is None else a_rows.numel()
    out = torch.empty(R, N if epi == EPI_NONE else N // 2, dtype=xp.dtype, device=xp.device)
    if R == 0:
        return out
    rows = avg_rows if avg_rows is not None else max(1, R // max(1, w.shape[0]))
    _sk_reserve(xp.device)
    torch.ops.mlop.grouped_gemm(out, xp, w, offsets, rows, epi, a_rows)
    return out
