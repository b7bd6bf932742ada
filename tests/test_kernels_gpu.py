"""Numerics of every gfx950 HIP kernel against the plain-PyTorch fp32 oracle
(``mlopamd.ops.reference``), on the MI355X."""
import math

import numpy as np
import pytest
import torch

from mlopamd import ops
from mlopamd.ops import reference as ref

pytestmark = pytest.mark.gpu
bf = torch.bfloat16


def close(a, b, atol=2e-2, rtol=2e-2):
    torch.testing.assert_close(a.float().cpu(), b.float().cpu(), atol=atol, rtol=rtol)


@pytest.mark.parametrize("M,H", [(1, 4096), (7, 4096), (33, 8192), (5, 1024), (3, 5120),
                                 (1027, 4096), (300, 1024), (259, 8192), (400, 5120)])
def test_rmsnorm(gpu, M, H):
    x = torch.randn(M, H, device=gpu, dtype=bf)
    w = (1 + 0.1 * torch.randn(H, device=gpu)).to(bf)
    close(ops.rmsnorm(x, w, 1e-5), ref.rmsnorm(x, w, 1e-5))


@pytest.mark.parametrize("M,H", [(1, 4096), (19, 4096), (4, 8192), (1030, 4096), (257, 2048), (300, 8192)])
def test_add_rmsnorm(gpu, M, H):
    x = torch.randn(M, H, device=gpu, dtype=bf)
    r = torch.randn(M, H, device=gpu, dtype=bf)
    w = (1 + 0.1 * torch.randn(H, device=gpu)).to(bf)
    y_ref, r_ref = ref.add_rmsnorm(x, r, w, 1e-5)
    r2 = r.clone()
    y = ops.add_rmsnorm(x, r2, w, 1e-5)
    close(r2, r_ref, atol=0, rtol=0)
    close(y, y_ref)


@pytest.mark.parametrize("M,I", [(1, 14336), (37, 14336), (8, 3584)])
def test_silu_mul(gpu, M, I):
    x = torch.randn(M, 2 * I, device=gpu, dtype=bf)
    close(ops.silu_mul(x), ref.silu_mul(x))


def test_embedding(gpu):
    table = torch.randn(1000, 256, device=gpu, dtype=bf)
    ids = torch.randint(0, 2000, (77,), device=gpu)
    close(ops.embedding(ids, table, 500), ref.embedding(ids, table, 500), atol=0, rtol=0)


@pytest.mark.parametrize("Hq,Hkv", [(32, 8), (8, 1), (16, 16)])
def test_rope_cache(gpu, Hq, Hkv):
    from mlopamd.models.layers import rope_table

    D, NB, BS, T = 128, 40, 16, 29
    cs = rope_table(D, 4096, 5e5, device=gpu)
    qkv = torch.randn(T, (Hq + 2 * Hkv) * D, device=gpu, dtype=bf)
    pos = torch.randint(0, 4000, (T,), device=gpu, dtype=torch.int32)
    slots = torch.randperm(NB * BS, device=gpu)[:T].to(torch.int32)
    slots[3] = -1
    kc = torch.zeros(NB, Hkv, BS, D, device=gpu, dtype=bf)
    vc = torch.zeros(NB, Hkv, BS, D, device=gpu, dtype=bf)
    kc2, vc2 = kc.clone(), vc.clone()
    q = ops.rope_cache(qkv, pos, cs, slots, kc, vc, Hq)
    q_ref = ref.rope_cache(qkv.cpu(), pos.cpu(), cs.cpu(), slots.cpu(), kc2.cpu(), vc2.cpu(), Hq)
    close(q, q_ref)
    # cache contents (ref wrote into the CPU copies)
    kr, vr = kc2.cpu(), vc2.cpu()
    ref.rope_cache(qkv.cpu(), pos.cpu(), cs.cpu(), slots.cpu(), kr, vr, Hq)
    close(kc, kr)
    close(vc, vr, atol=0, rtol=0)


@pytest.mark.parametrize("M,Hq,Hkv", [(300, 32, 8), (1024, 32, 8), (2048, 32, 8), (3000, 32, 8),
                                      (600, 8, 1), (12, 32, 8), (16, 32, 8), (24, 32, 8), (48, 32, 8),
                                      (16, 8, 1)])
def test_qkv_rope_cache_fused(gpu, M, Hq, Hkv):
    """QKV GEMM with RoPE + paged K/V stores in its epilogue (EPI_ROPE; the ping-pong
    256x256 kernel at M=2048/3000, the 256x128 kernel otherwise; decode-size M: split-K slabs
    whose reduce is fused into the RoPE + cache kernel) vs fp32 GEMM + rope_cache."""
    from mlopamd.models.layers import rope_table

    D, K, BS = 128, 4096, 16
    N = (Hq + 2 * Hkv) * D
    NB = M // BS + 8
    ops._sk_reserve(torch.device(gpu))  # M = 2048 / 3000: stream-K tail (192 / 288 tiles)
    cs = rope_table(D, 8192, 5e5, device=gpu)
    x = torch.randn(M, K, device=gpu, dtype=bf)
    w = (0.02 * torch.randn(N, K, device=gpu)).to(bf)
    pos = torch.randint(0, 8000, (M,), device=gpu, dtype=torch.int32)
    slots = torch.randperm(NB * BS, device=gpu)[:M].to(torch.int32)
    slots[5] = -1
    slots[M - 1] = -1
    prev = torch.ops.mlop.gemm_small_tile()
    if M <= 64:  # the 64-column small-M tiles split K at these N: the slab-fed RoPE kernel
        torch.ops.mlop.gemm_small_tile(64)
    try:
        assert torch.ops.mlop.gemm_rope_supported(M, N, K)
        kc = torch.zeros(NB, Hkv, BS, D, device=gpu, dtype=bf)
        vc = torch.zeros(NB, Hkv, BS, D, device=gpu, dtype=bf)
        q = torch.empty(M, Hq, D, device=gpu, dtype=bf)
        assert torch.ops.mlop.gemm_rope_cache(q, kc, vc, x, w, pos, cs, slots)
        qkv_ref = (x.float() @ w.float().t()).to(bf).cpu()
        kr, vr = torch.zeros_like(kc).cpu(), torch.zeros_like(vc).cpu()
        q_ref = ref.rope_cache(qkv_ref, pos.cpu(), cs.cpu(), slots.cpu(), kr, vr, Hq)
        close(q, q_ref)
        close(kc, kr)
        close(vc, vr)
    finally:
        torch.ops.mlop.gemm_small_tile(prev)
    # the wrapper (autotuned fused vs hipBLASLt + rope_cache; default small-M tiles) agrees too
    q2 = ops.qkv_rope_cache(x, w, pos, cs, slots, kc, vc, Hq)
    close(q2, q_ref)


class Meta:
    pass


def make_meta(gpu, q_lens, ctx_lens, Hkv, G, NB, part_tokens=None, nparts=1, shuffle_rows=True,
              flash_min_q=1 << 30):
    """Rows with q_len >= flash_min_q get flash-prefill tiles (128/G tokens, latest first)."""
    from mlopamd.runtime.attn_meta import plan_partitions

    S = len(q_lens)
    MB = max(1, max((c + 15) // 16 for c in ctx_lens))
    rows = np.random.permutation(S + 3)[:S] if shuffle_rows else np.arange(S)
    R = S + 3
    bt = np.zeros((R, MB), dtype=np.int32)
    pages = np.random.permutation(np.arange(1, NB))
    p = 0
    for i, c in enumerate(ctx_lens):
        n = (c + 15) // 16
        bt[rows[i], :n] = pages[p:p + n]
        p += n
    qt = 16 // G
    q_start = np.zeros(R, np.int32); q_len = np.zeros(R, np.int32); ctx = np.zeros(R, np.int32)
    ts, tq, pts, ptq = [], [], [], []
    pqt = 128 // G
    t = 0
    for i in range(S):
        r = rows[i]
        q_start[r], q_len[r], ctx[r] = t, q_lens[i], ctx_lens[i]
        if q_lens[i] >= flash_min_q and G <= 8:
            n = (q_lens[i] + pqt - 1) // pqt
            pts += [r] * n
            ptq += list(range((n - 1) * pqt, -1, -pqt))
        else:
            nt = (q_lens[i] + qt - 1) // qt
            ts += [r] * nt
            tq += list(range(0, nt * qt, qt))
        t += q_lens[i]
    m = Meta()
    d = lambda a: torch.tensor(np.asarray(a), dtype=torch.int32, device=gpu)  # noqa: E731
    m.block_tables, m.q_start, m.q_len, m.ctx_len = d(bt), d(q_start), d(q_len), d(ctx)
    m.tile_seq, m.tile_q0 = d(np.asarray(ts, np.int32)), d(np.asarray(tq, np.int32))
    m.ptile_seq, m.ptile_q0 = d(np.asarray(pts, np.int32)), d(np.asarray(ptq, np.int32))
    if part_tokens is None:
        part_tokens, nparts = plan_partitions(len(ts), Hkv, max(ctx_lens))
    m.part_tokens, m.nparts = part_tokens, nparts
    m.part_o = torch.empty(len(ts) * Hkv * nparts * 16 * 128, device=gpu)
    m.part_ml = torch.empty(len(ts) * Hkv * nparts * 16 * 2, device=gpu)
    return m, t


@pytest.fixture(params=[(0, 0), (3 * 64, 0), (3 * 64, 1), (64, 1)], ids=["grid", "persist3", "stream3", "stream1"])
def flash_persist(request):
    """One workgroup per flash item, or the persistent grid forced to 3 slots per kv head (every
    slot walks several boustrophedon rounds, a partial last one included), per tile or as one
    cross-tile stream of K / V pairs and Q (flash_stream); stream1: ONE slot per kv head streams
    every tile of the launch, one-pair tiles included."""
    persist, stream = request.param
    prev, prev_s = torch.ops.mlop.flash_persist(-1), torch.ops.mlop.flash_stream(-1)
    torch.ops.mlop.flash_persist(persist)
    torch.ops.mlop.flash_stream(stream)
    yield request.param
    torch.ops.mlop.flash_persist(prev)
    torch.ops.mlop.flash_stream(prev_s)


@pytest.mark.parametrize("Hq,Hkv", [(32, 8), (8, 1), (64, 8), (16, 16), (32, 16), (16, 8)])
@pytest.mark.parametrize("q_lens,ctx_lens", [
    ([1, 40, 200, 17], [1, 40, 200, 17]),            # fresh prompts, partial last tiles
    ([300, 1, 130], [1500, 700, 130]),               # chunked prefill continuing a context + a decode row
    ([1024], [1024]),                                # one long prompt (many causal tiles)
])
def test_flash_prefill(gpu, Hq, Hkv, q_lens, ctx_lens, flash_persist):
    """K7 flash-prefill tiles (with the decode kernel on the short rows of the
    same launch) against the fp32 reference attention."""
    torch.manual_seed(0)
    np.random.seed(0)
    G = Hq // Hkv
    NB = sum((c + 15) // 16 for c in ctx_lens) + 8
    kc = torch.randn(NB, Hkv, 16, 128, device=gpu, dtype=bf)
    vc = torch.randn(NB, Hkv, 16, 128, device=gpu, dtype=bf)
    m, T = make_meta(gpu, q_lens, ctx_lens, Hkv, G, NB, flash_min_q=17)
    assert m.ptile_seq.numel() > 0
    q = torch.randn(T, Hq, 128, device=gpu, dtype=bf)
    out = ops.paged_attention(q, kc, vc, m)
    close(out, ref.paged_attention(q, kc, vc, m), atol=2e-2, rtol=2e-2)


def test_flash_prefill_growing_scores(gpu):
    """Scores whose row max keeps growing along the keys (K scaled up page by page): the
    deferred rescale (threshold 2^8) fires again and again, the path random data rarely takes."""
    torch.manual_seed(1)
    np.random.seed(1)
    Hq, Hkv, L = 32, 8, 700
    NB = (L + 15) // 16 + 8
    vc = torch.randn(NB, Hkv, 16, 128, device=gpu, dtype=bf)
    m, T = make_meta(gpu, [L], [L], Hkv, Hq // Hkv, NB, flash_min_q=17)
    # positive K growing with the LOGICAL page index (through the block table): q . k grows
    # along the keys of the sequence
    row = int(torch.nonzero(m.q_len == L)[0, 0])
    n = (L + 15) // 16
    pages = m.block_tables[row, :n].long()
    kc = torch.zeros(NB, Hkv, 16, 128, device=gpu)
    kc[pages] = torch.randn(n, Hkv, 16, 128, device=gpu).abs() * torch.linspace(0.2, 3.0, n, device=gpu).view(n, 1, 1, 1)
    kc = kc.to(bf)
    q = (torch.rand(T, Hq, 128, device=gpu) + 0.5).to(bf)
    out = ops.paged_attention(q, kc, vc, m)
    close(out, ref.paged_attention(q, kc, vc, m), atol=2e-2, rtol=2e-2)


@pytest.mark.parametrize("Hq,Hkv", [(32, 8), (8, 1), (64, 8), (16, 16)])
@pytest.mark.parametrize("case", ["decode", "prefill", "mixed", "split", "split_fused"])
def test_paged_attention(gpu, Hq, Hkv, case, attn_fused_all):
    torch.manual_seed(0)
    np.random.seed(0)
    G = Hq // Hkv
    NB = 400
    if case == "decode":
        q_lens, ctx_lens = [1] * 9, [1, 15, 16, 17, 100, 511, 512, 700, 1300]
    elif case == "prefill":
        q_lens = [1, 7, 64, 200]
        ctx_lens = list(q_lens)
    elif case == "mixed":
        q_lens, ctx_lens = [1, 37, 1, 130], [300, 90, 64, 1000]
    else:  # forced split-KV with a reduce pass
        q_lens, ctx_lens = [1, 1, 3], [1500, 33, 900]
    kc = torch.randn(NB, Hkv, 16, 128, device=gpu, dtype=bf)
    vc = torch.randn(NB, Hkv, 16, 128, device=gpu, dtype=bf)
    kw = dict(part_tokens=256, nparts=6) if case.startswith("split") else {}
    m, T = make_meta(gpu, q_lens, ctx_lens, Hkv, G, NB, **kw)
    q = torch.randn(T, Hq, 128, device=gpu, dtype=bf)
    exp = ref.paged_attention(q, kc, vc, m)
    if case == "split_fused":
        # in-launch combine by the last-arriving partition; the tickets must come back
        # re-armed (all zero) after every launch, so repeated launches stay correct
        m.part_sem = torch.zeros(m.tile_seq.numel() * Hkv, dtype=torch.int32, device=gpu)
        for _ in range(3):
            out = ops.paged_attention(q, kc, vc, m)
            close(out, exp, atol=2e-2, rtol=2e-2)
            assert int(m.part_sem.abs().sum()) == 0
        return
    out = ops.paged_attention(q, kc, vc, m)
    close(out, exp, atol=2e-2, rtol=2e-2)


@pytest.mark.parametrize("fused", [False, True])
def test_paged_attention_padded_bucket(gpu, fused, attn_fused_all):
    """Graph-bucket padding rows (q_len 1, ctx 0) under forced split-KV: both combine
    paths (second-launch reduce and in-launch last-ticket combine) must write a zero
    row there, not leave the buffer's old contents (NaN here) for o_proj / MoE routing."""
    torch.manual_seed(0)
    np.random.seed(0)
    Hq, Hkv, NB = 32, 8, 400
    q_lens, ctx_lens = [1, 1, 3, 1, 1], [1500, 33, 900, 0, 0]
    kc = torch.randn(NB, Hkv, 16, 128, device=gpu, dtype=bf)
    vc = torch.randn(NB, Hkv, 16, 128, device=gpu, dtype=bf)
    m, T = make_meta(gpu, q_lens, ctx_lens, Hkv, Hq // Hkv, NB, part_tokens=256, nparts=6,
                     shuffle_rows=False)
    if fused:
        m.part_sem = torch.zeros(m.tile_seq.numel() * Hkv, dtype=torch.int32, device=gpu)
    q = torch.randn(T, Hq, 128, device=gpu, dtype=bf)
    exp = ref.paged_attention(q, kc, vc, m)
    for _ in range(2):
        out = torch.full_like(q, float("nan"))
        ops.paged_attention(q, kc, vc, m, out=out)
        assert torch.isfinite(out).all()
        assert (out[-2:] == 0).all()
        close(out, exp, atol=2e-2, rtol=2e-2)
        if fused:
            assert int(m.part_sem.abs().sum()) == 0


def test_attention_spike_rescale(gpu):
    """Force the online-softmax rescale branch: a late key dominates."""
    Hq, Hkv = 32, 8
    kc = 0.1 * torch.randn(100, Hkv, 16, 128, device=gpu, dtype=bf)
    vc = torch.randn(100, Hkv, 16, 128, device=gpu, dtype=bf)
    m, T = make_meta(gpu, [1, 4], [600, 700], Hkv, 4, 100, shuffle_rows=False)
    q = torch.randn(T, Hq, 128, device=gpu, dtype=bf)
    bt = m.block_tables.cpu()
    page = int(bt[0, 30])
    kc[page, :, 5, :] = 3.0 * q[0, ::4, :].to(bf)  # key 485 aligned with the query
    out = ops.paged_attention(q, kc, vc, m)
    close(out, ref.paged_attention(q, kc, vc, m), atol=3e-2, rtol=3e-2)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("n,V", [(1, 128256), (2, 128256), (64, 128256), (5, 32000), (100, 32000), (3, 1000),
                                 (2, 1003), (1, 16040)])
def test_argmax(gpu, n, V, dtype):
    x = torch.randn(n, V, device=gpu).to(dtype)
    if V % (8 if dtype == torch.bfloat16 else 4):
        # rows that are not 16-B aligned are refused loudly, never read misaligned
        with pytest.raises(RuntimeError, match="16-B aligned"):
            ops.argmax(x)
        return
    if dtype == torch.bfloat16:
        x[:, 7] = x.max()  # exact ties (common in bf16): the smallest index wins, as in torch
    assert torch.equal(ops.argmax(x).cpu(), x.float().argmax(-1).cpu())


@pytest.mark.parametrize("n,V", [(16, 32000), (4, 128256), (64, 32000), (8, 1000)])
def test_sample_matches_reference(gpu, n, V):
    """n < 64: per-slice top-K pre-selection (16 workgroups per row) + the draw over the
    candidates; n = 64: the single-stage kernel; rows with top_k = 0: the full-vocabulary
    kernel (softmax over the WHOLE row, top-p over the full mass); same uniforms as the reference.

    Exact, tie-safe check of EVERY row: the drawn token must be the one whose interval
    [c_{j-1}, c_j) of the fp64 reference CDF holds u (candidates in value order for top-k rows;
    the nucleus in vocabulary order for full rows).  Only when u or the top-p cut lies within
    1e-5 of an interval edge -- where fp32 summation order legitimately decides -- is the
    neighbouring candidate accepted as well."""
    torch.manual_seed(1)
    x = 3 * torch.randn(n, V, device=gpu)
    temps = torch.tensor([0.0, 0.7, 1.0, 1.3] * (n // 4), device=gpu)
    ks = torch.tensor([0, 1, 50, 0] * (n // 4), dtype=torch.int32, device=gpu)
    ps = torch.tensor([1.0, 1.0, 0.9, 0.5] * (n // 4), device=gpu)
    u = torch.rand(n, device=gpu)
    got = ops.sample(x, temps, ks, ps, u).cpu()
    from mlopamd.runtime.sampler import MAX_TOP_K

    eps = 1e-5
    kmax = min(MAX_TOP_K, V)
    xd = x.cpu().double()
    vals, idx = torch.topk(xd, kmax, dim=-1)
    for i in range(n):
        if float(temps[i]) <= 0 or int(ks[i]) == 1:  # greedy rows: exact argmax
            assert int(got[i]) == int(idx[i, 0]), i
            continue
        pp, ui, T = float(ps[i]), float(u[i]), float(temps[i])
        if int(ks[i]) == 0:  # the whole vocabulary
            w = torch.exp((xd[i] - xd[i].max()) / T)
            order = torch.sort(-xd[i], stable=True).indices
            cum = torch.cumsum(w[order], 0) / w.sum()
            keep0 = int((cum < pp).sum()) + 1 if pp < 1 else V
            keeps = {min(keep0, V)} | {kk for kk in (keep0 - 1, keep0 + 1)
                                       if pp < 1 and 1 <= kk <= V and abs(float(cum[kk - 1]) - pp) < eps}
            ok = False
            for keep in keeps:
                nuc = torch.zeros(V, dtype=torch.bool)
                nuc[order[:keep]] = True
                if not nuc[int(got[i])]:
                    continue
                c = torch.cumsum(w * nuc, 0) / (w * nuc).sum()
                j = int(got[i])
                lo = 0.0 if j == 0 else float(c[j - 1])
                ok |= lo - eps <= ui <= float(c[j]) + eps
            assert ok, (i, int(got[i]), ui)
            continue
        k = min(int(ks[i]), kmax)
        pr = torch.softmax(vals[i, :k] / T, dim=-1)
        c = torch.cumsum(pr, dim=-1)
        keeps = {k}
        if pp < 1.0:
            keep = min(int((c < pp).sum()) + 1, k)
            keeps = {keep} | {kk for kk in (keep - 1, keep + 1) if 1 <= kk <= k and abs(float(c[kk - 1]) - pp) < eps}
        ok = False
        for keep in keeps:
            cc = torch.cumsum(pr[:keep] / c[keep - 1], dim=-1)
            pos = (idx[i, :keep] == int(got[i])).nonzero()
            if pos.numel() == 0:
                continue
            j = int(pos[0])
            lo = 0.0 if j == 0 else float(cc[j - 1])
            hi = 1.0 if j == keep - 1 else float(cc[j])
            ok |= lo - eps <= ui <= hi + eps
        assert ok, (i, int(got[i]), ui)


def test_sample_full_vocab_distribution(gpu):
    """temperature > 0, top_k = 0, top_p = 1 samples the UNTRUNCATED softmax: over a 4096-token
    vocabulary whose logits are flat up to a +-0.3 ramp, 3/4 of the mass lies outside the top
    1024 logits (a 1024-candidate sampler would never draw there).  8192 draws; the empirical
    frequencies of 8 equal-width index bands match the fp64 softmax within 4 sigma.  Also the
    top_p = 0.5 nucleus: no draw outside the smallest prefix holding half the mass."""
    V, n = 4096, 8192
    torch.manual_seed(3)
    row = torch.linspace(-0.3, 0.3, V, device=gpu)[torch.randperm(V, device=gpu)]
    x = row.expand(n, V).contiguous()
    temps = torch.ones(n, device=gpu)
    ks = torch.zeros(n, dtype=torch.int32, device=gpu)
    got = ops.sample(x, temps, ks, torch.ones(n, device=gpu), torch.rand(n, device=gpu)).cpu()
    p = torch.softmax(row.double().cpu(), 0)
    top1024 = set(torch.topk(row.cpu(), 1024).indices.tolist())
    outside = sum(int(t) not in top1024 for t in got.tolist()) / n
    p_out = 1 - float(p[list(top1024)].sum())
    assert abs(outside - p_out) < 4 * (p_out * (1 - p_out) / n) ** 0.5 + 1e-3, (outside, p_out)
    band = got // (V // 8)
    for b in range(8):
        pb = float(p[b * V // 8:(b + 1) * V // 8].sum())
        fb = float((band == b).float().mean())
        assert abs(fb - pb) < 4 * (pb * (1 - pb) / n) ** 0.5 + 1e-3, (b, fb, pb)
    got = ops.sample(x, temps, ks, torch.full((n,), 0.5, device=gpu), torch.rand(n, device=gpu)).cpu()
    order = torch.sort(-row.double().cpu(), stable=True).indices
    keep = int((torch.cumsum(p[order], 0) < 0.5).sum()) + 1
    assert set(got.tolist()) <= set(order[:keep + 1].tolist())


def test_sampler_seed_reproducible(gpu):
    """SamplingParams.seed: the same (seed, output position) draws the same uniform in any batch."""
    from mlopamd.runtime.sampler import Sampler, SamplingParams

    torch.manual_seed(4)
    x = torch.randn(6, 32000, device=gpu)
    mk = lambda s: SamplingParams(temperature=1.0, top_k=0, seed=s)  # noqa: E731
    a = Sampler(gpu, seed=1)(x, [mk(7), mk(8), mk(None), mk(7), mk(9), mk(7)], gen_index=[3, 3, 0, 3, 0, 4])
    b = Sampler(gpu, seed=2)(x[[3, 0, 1]], [mk(7), mk(7), mk(8)], gen_index=[3, 3, 3])
    assert int(a[0]) == int(b[1]) and int(a[1]) == int(b[2]) and int(a[3]) == int(b[0])


@pytest.mark.parametrize("M,N,K", [(1, 4096, 4096), (7, 6144, 4096), (64, 4096, 14336),
                                   (128, 1280, 1024), (256, 4096, 4096), (256, 6144, 4096),
                                   (300, 1024, 512), (1500, 4096, 4096), (1000, 16032, 1024),
                                   (2048, 6144, 4096), (1100, 4352, 1024), (4096, 4096, 64), (3000, 1000, 512)])
def test_gemm(gpu, M, N, K):
    torch.manual_seed(M + N)
    x = torch.randn(M, K, device=gpu, dtype=bf)
    w = (0.05 * torch.randn(N, K, device=gpu)).to(bf)
    ops.GEMM_BACKEND = "mlop"  # the hand-written kernel, whatever the autotuner would pick
    try:
        y = ops.gemm(x, w)
    finally:
        ops.GEMM_BACKEND = ops.GEMM_BACKEND_DEFAULT
    exp = (x.float() @ w.float().t())
    close(y, exp, atol=3e-2 * exp.abs().max().item() / 10 + 1e-2, rtol=2e-2)


@pytest.mark.parametrize("M,N,K,epi", [
    (2040, 28672, 4096, 1),   # 896 tiles: 768 data-parallel + 128 tail tiles in 2 halves (gate_up, SiLU)
    (4352, 4096, 14336, 0),   # 272 tiles: 16 tail tiles x 224 K-tiles in 8 ranges (re-read sum path)
    (3072, 6144, 4096, 0),    # 288 tiles: 32 tail tiles in 4 ranges of 16 K-tiles
    (2100, 8320, 2048, 0),    # ragged M and N: 297 tiles, 41 tail tiles in 2 halves
])
def test_gemm_stream_k(gpu, pp_variant, M, N, K, epi):
    """Stream-K tail of the ping-pong GEMM (partial tiles through fp32 slots, ticket
    counters, last-arriver fixup + epilogue): vs fp32 matmul, three launches in a row
    (the counters re-arm), and against the data-parallel grid of the same kernel."""
    torch.manual_seed(M + K)
    ops._sk_reserve(torch.device(gpu))
    assert torch.ops.mlop.gemm_sk_workgroups(M, N, K) > 0
    x = torch.randn(M, K, device=gpu, dtype=bf)
    w = (0.05 * torch.randn(N, K, device=gpu)).to(bf)
    exp = x.float() @ w.float().t()
    if epi:
        exp = ref.silu_mul(ops.deinterleave_cols(exp.to(bf)))
    ops.GEMM_BACKEND = "mlop"
    try:
        outs = [ops.gemm(x, w, epi=epi) for _ in range(3)]
        prev = torch.ops.mlop.gemm_sk_mode(-1)
        torch.ops.mlop.gemm_sk_mode(0)
        dp = ops.gemm(x, w, epi=epi)
        torch.ops.mlop.gemm_sk_mode(prev)
    finally:
        ops.GEMM_BACKEND = ops.GEMM_BACKEND_DEFAULT
    tol = 3e-2 * exp.abs().max().item() / 10 + 1e-2
    for y in outs + [dp]:
        close(y, exp, atol=tol, rtol=2e-2)
    close(outs[0], outs[2], atol=0, rtol=0)  # deterministic: fixed slot order in the fixup


@pytest.mark.parametrize("M", [1, 2, 3, 4, 5, 8])
@pytest.mark.parametrize("N,K", [(4096, 4096), (6144, 4096), (4096, 14336), (1280, 8192), (8192, 1024),
                                 (8192, 3584), (16, 1024)])
def test_gemv(gpu, M, N, K):
    """K2 skinny GEMV (gemv.hip, M <= 4; M = 5 / 8 take the MFMA tiles): wave-per-row-pair
    (N >= 4096) and the 4-waves-split-K form (N = 1280 / 16: 70B TP=8 shards, tiny N), K
    not a multiple of the unrolled stride (1024, 3584); vs fp32 matmul."""
    torch.manual_seed(M * 7 + N + K)
    x = torch.randn(M, K, device=gpu, dtype=bf)
    w = (0.05 * torch.randn(N, K, device=gpu)).to(bf)
    if M <= 4:
        assert torch.ops.mlop.gemm_workspace(M, N, K, 0) == 0  # no split-K slabs on this path
    y = torch.empty(M, N, device=gpu, dtype=bf)
    nws = torch.ops.mlop.gemm_workspace(M, N, K, 0)
    torch.ops.mlop.gemm(y, x, w, torch.empty(max(nws, 0), device=gpu), 0)
    exp = x.float() @ w.float().t()
    close(y, exp, atol=2e-2 * exp.abs().max().item() / 10 + 1e-2, rtol=2e-2)


@pytest.mark.parametrize("M", [5, 13, 16, 24, 32, 48, 64])
@pytest.mark.parametrize("tile", [1, 32, 64])
@pytest.mark.parametrize("N,K,epi", [(6144, 4096, 0), (4096, 14336, 0), (7168, 4096, 1), (1280, 8192, 0),
                                     (28672, 4096, 1)])
def test_gemm_small_tiles(gpu, M, tile, N, K, epi):
    """Row-fitted LDS-DMA tiles for M <= 64 (gemm.hip plan, ``gemm_small_tile``): BM 16 / 32 / 64
    by the batch, BN 32 / 64 (1 = per shape: 8- / 6-deep rings at BM 16), split-K slabs on
    narrow N; plain, SiLU-mul and the fused add + RMSNorm reduce; vs fp32 matmul."""
    torch.manual_seed(M * 7 + tile + N)
    x = torch.randn(M, K, device=gpu, dtype=bf)
    if epi:
        g = (0.05 * torch.randn(N // 2, K, device=gpu)).to(bf)
        u = (0.05 * torch.randn(N // 2, K, device=gpu)).to(bf)
        w = ops.interleave_gate_up(g, u)
        exp = ref.silu_mul((x.float() @ torch.cat([g, u]).float().t()).to(bf))
    else:
        w = (0.05 * torch.randn(N, K, device=gpu)).to(bf)
        exp = x.float() @ w.float().t()
    prev = torch.ops.mlop.gemm_small_tile()
    torch.ops.mlop.gemm_small_tile(tile)
    try:
        y = torch.empty(M, N // 2 if epi else N, device=gpu, dtype=bf)
        nws = torch.ops.mlop.gemm_workspace(M, N, K, epi)
        torch.ops.mlop.gemm(y, x, w, torch.full((max(nws, 1),), float("nan"), device=gpu), epi)
        close(y, exp, atol=3e-2 * exp.abs().max().item() / 10 + 1e-2, rtol=2e-2)
        if not epi and nws:  # split-K: the residual add + RMSNorm reduce on the same slabs
            res = torch.randn(M, N, device=gpu, dtype=bf)
            nw = (1 + 0.1 * torch.randn(N, device=gpu)).to(bf)
            e_out, e_res = ref.add_rmsnorm(exp.to(bf), res, nw, 1e-5)
            out = torch.empty(M, N, device=gpu, dtype=bf)
            assert torch.ops.mlop.gemm_add_rmsnorm(out, res, x, w, nw, torch.empty(nws, device=gpu), 1e-5)
            close(res, e_res, atol=3e-2, rtol=2e-2)
            close(out, e_out, atol=5e-2, rtol=3e-2)
    finally:
        torch.ops.mlop.gemm_small_tile(prev)


@pytest.mark.parametrize("M", [5, 8, 16, 17, 32, 40, 64])
@pytest.mark.parametrize("N,K,epi", [(6144, 4096, 0), (4096, 14336, 0), (7168, 4096, 1), (28672, 4096, 1),
                                     (1280, 8192, 0)])
def test_mid_m_gemm(gpu, M, N, K, epi):
    """Decode projections above the GEMV's rows (4 < M <= 64): the row-fitted LDS-DMA MFMA tiles
    with their split-K fp32 slabs reduced by gemm.hip (plain / SiLU-mul epilogue); ragged M
    (17, 40: clamped A rows); NaN-filled workspace (every slab element must be written)."""
    torch.manual_seed(M * 13 + N + K + epi)
    x = torch.randn(M, K, device=gpu, dtype=bf)
    if epi:
        g = (0.05 * torch.randn(N // 2, K, device=gpu)).to(bf)
        u = (0.05 * torch.randn(N // 2, K, device=gpu)).to(bf)
        w = ops.interleave_gate_up(g, u)
        exp = ref.silu_mul((x.float() @ torch.cat([g, u]).float().t()).to(bf))
    else:
        w = (0.05 * torch.randn(N, K, device=gpu)).to(bf)
        exp = x.float() @ w.float().t()
    y = torch.empty(M, N // 2 if epi else N, device=gpu, dtype=bf)
    nws = torch.ops.mlop.gemm_workspace(M, N, K, epi)
    torch.ops.mlop.gemm(y, x, w, torch.full((max(nws, 1),), float("nan"), device=gpu), epi)
    close(y, exp, atol=3e-2 * exp.abs().max().item() / 10 + 1e-2, rtol=2e-2)


@pytest.mark.parametrize("M", [1, 2, 4])
@pytest.mark.parametrize("I,K", [(14336, 4096), (3584, 8192)])
def test_gemv_silu_mul(gpu, M, I, K):
    torch.manual_seed(M + I)
    x = torch.randn(M, K, device=gpu, dtype=bf)
    g = (0.05 * torch.randn(I, K, device=gpu)).to(bf)
    u = (0.05 * torch.randn(I, K, device=gpu)).to(bf)
    w = ops.interleave_gate_up(g, u)
    ops.GEMM_BACKEND = "mlop"
    try:
        y = ops.gemm(x, w, epi=ops.EPI_SILU_MUL)
    finally:
        ops.GEMM_BACKEND = ops.GEMM_BACKEND_DEFAULT
    gu = (x.float() @ torch.cat([g, u]).float().t()).to(bf)
    close(y, ref.silu_mul(gu), atol=3e-2, rtol=3e-2)


@pytest.mark.parametrize("consecutive", [False, True])
def test_qkv_rope_fused_in_graph(gpu, consecutive):
    """Large-M fused QKV+RoPE (K rotated, K and V rows stored into their token-major pages
    from the GEMM epilogue) captured in a hipGraph and replayed with new positions / slots:
    replay == eager reference.  Consecutive slots = a prefill chunk; random = decode rows."""
    from mlopamd.models.layers import rope_table

    M, Hq, Hkv, D, K, BS = 1024, 32, 8, 128, 4096, 16
    N = (Hq + 2 * Hkv) * D
    NB = M // BS + 8
    ops._sk_reserve(torch.device(gpu))
    cs = rope_table(D, 8192, 5e5, device=gpu)
    x = torch.randn(M, K, device=gpu, dtype=bf)
    w = (0.02 * torch.randn(N, K, device=gpu)).to(bf)
    pos = torch.zeros(M, device=gpu, dtype=torch.int32)
    slots = torch.zeros(M, device=gpu, dtype=torch.int32)
    kc = torch.zeros(NB, Hkv, BS, D, device=gpu, dtype=bf)
    vc = torch.zeros(NB, Hkv, BS, D, device=gpu, dtype=bf)
    q = torch.empty(M, Hq, D, device=gpu, dtype=bf)
    assert torch.ops.mlop.gemm_rope_supported(M, N, K)
    torch.ops.mlop.gemm_rope_cache(q, kc, vc, x, w, pos, cs, slots)  # warm-up outside capture
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        torch.ops.mlop.gemm_rope_cache(q, kc, vc, x, w, pos, cs, slots)
    new_slots = (torch.arange(M, device=gpu) + 3 * BS) if consecutive else torch.randperm(NB * BS, device=gpu)[:M]
    slots.copy_(new_slots.to(torch.int32))
    slots[7] = -1
    pos.copy_(torch.randint(0, 8000, (M,), device=gpu, dtype=torch.int32))
    kc.zero_()
    vc.zero_()
    g.replay()
    torch.cuda.synchronize()
    qkv_ref = (x.float() @ w.float().t()).to(bf).cpu()
    kr, vr = torch.zeros_like(kc).cpu(), torch.zeros_like(vc).cpu()
    q_ref = ref.rope_cache(qkv_ref, pos.cpu(), cs.cpu(), slots.cpu(), kr, vr, Hq)
    close(q, q_ref)
    close(kc, kr)
    close(vc, vr)


@pytest.mark.parametrize("M,Hq,Hkv", [(1, 32, 8), (3, 32, 8), (4, 32, 8), (2, 8, 1), (4, 64, 8)])
def test_gemv_rope_cache(gpu, M, Hq, Hkv):
    """Decode QKV GEMV with RoPE + paged K/V stores in its epilogue (EPI_ROPE at M <= 8)."""
    from mlopamd.models.layers import rope_table

    D, K, BS, NB = 128, 4096, 16, 64
    N = (Hq + 2 * Hkv) * D
    cs = rope_table(D, 8192, 5e5, device=gpu)
    x = torch.randn(M, K, device=gpu, dtype=bf)
    w = (0.02 * torch.randn(N, K, device=gpu)).to(bf)
    pos = torch.randint(0, 8000, (M,), device=gpu, dtype=torch.int32)
    slots = torch.randperm(NB * BS, device=gpu)[:M].to(torch.int32)
    if M > 2:
        slots[1] = -1  # padding row: no cache write
    assert torch.ops.mlop.gemm_rope_supported(M, N, K)
    kc = torch.zeros(NB, Hkv, BS, D, device=gpu, dtype=bf)
    vc = torch.zeros(NB, Hkv, BS, D, device=gpu, dtype=bf)
    q = torch.empty(M, Hq, D, device=gpu, dtype=bf)
    assert torch.ops.mlop.gemm_rope_cache(q, kc, vc, x, w, pos, cs, slots)
    qkv_ref = (x.float() @ w.float().t()).to(bf).cpu()
    kr, vr = torch.zeros_like(kc).cpu(), torch.zeros_like(vc).cpu()
    q_ref = ref.rope_cache(qkv_ref, pos.cpu(), cs.cpu(), slots.cpu(), kr, vr, Hq)
    close(q, q_ref)
    close(kc, kr)
    close(vc, vr)


@pytest.mark.parametrize("M,N,K", [(1, 4096, 4096), (64, 4096, 14336), (256, 4096, 4096), (256, 4096, 14336)])
def test_gemm_add_rmsnorm(gpu, M, N, K):
    torch.manual_seed(K)
    x = torch.randn(M, K, device=gpu, dtype=bf)
    w = (0.02 * torch.randn(N, K, device=gpu)).to(bf)
    res = torch.randn(M, N, device=gpu, dtype=bf)
    nw = (1 + 0.1 * torch.randn(N, device=gpu)).to(bf)
    y = (x.float() @ w.float().t()).to(bf)
    exp_out, exp_res = ref.add_rmsnorm(y, res, nw, 1e-5)
    for backend in ("mlop", "hipblaslt"):
        ops.GEMM_BACKEND = backend
        try:
            r2 = res.clone()
            out = ops.gemm_add_rmsnorm(x, w, r2, nw, 1e-5)
        finally:
            ops.GEMM_BACKEND = ops.GEMM_BACKEND_DEFAULT
        close(r2, exp_res, atol=3e-2, rtol=2e-2)
        close(out, exp_out, atol=5e-2, rtol=3e-2)


@pytest.mark.parametrize("M,I,K", [(1, 14336, 4096), (37, 3584, 4096), (256, 14336, 4096), (900, 512, 256),
                                   (2048, 14336, 4096), (1300, 640, 512)])
def test_gemm_silu_mul(gpu, M, I, K):
    torch.manual_seed(I)
    x = torch.randn(M, K, device=gpu, dtype=bf)
    g = (0.05 * torch.randn(I, K, device=gpu)).to(bf)
    u = (0.05 * torch.randn(I, K, device=gpu)).to(bf)
    w = ops.interleave_gate_up(g, u)
    ops.GEMM_BACKEND = "mlop"
    try:
        y = ops.gemm(x, w, epi=ops.EPI_SILU_MUL)
    finally:
        ops.GEMM_BACKEND = ops.GEMM_BACKEND_DEFAULT
    gu = (x.float() @ torch.cat([g, u]).float().t()).to(bf)
    close(y, ref.silu_mul(gu), atol=3e-2, rtol=3e-2)


@pytest.fixture(params=[(0, 0), (1, 0), (2, 0), (2, 1), (2, 2)],
                ids=["spill", "balanced", "balanced16", "expert_major", "order_auto"])
def grouped_balance(request):
    """An expert over several 256-row m-tiles: full tiles + a spill tile, or equal row ranges
    (gemm_grouped_balance); tiles in the slot-fastest or the expert-major order
    (gemm_grouped_order)."""
    bal, order = request.param
    prev, prev_o = torch.ops.mlop.gemm_grouped_balance(-1), torch.ops.mlop.gemm_grouped_order(-1)
    torch.ops.mlop.gemm_grouped_balance(bal)
    torch.ops.mlop.gemm_grouped_order(order)
    yield request.param
    torch.ops.mlop.gemm_grouped_balance(prev)
    torch.ops.mlop.gemm_grouped_order(prev_o)


@pytest.mark.parametrize("rows", [[520, 700, 0, 613], [1024, 1024, 1024, 1024], [512, 3, 900, 257]])
@pytest.mark.parametrize("epi", [0, 1])
def test_grouped_gemm_large_groups(gpu, rows, epi, grouped_balance):
    """>= 512 rows per expert on average: the grouped ping-pong 256x256 kernel; ragged,
    empty and tiny groups included; vs per-group fp32 matmul."""
    torch.manual_seed(sum(rows))
    E, K, N = len(rows), 512, 1024
    off = torch.tensor([0] + list(np.cumsum(rows)), device=gpu, dtype=torch.int32)
    Mt = int(off[-1])
    x = torch.randn(Mt, K, device=gpu, dtype=bf)
    w = (0.05 * torch.randn(E, N, K, device=gpu)).to(bf)
    y = ops.grouped_gemm(x, w, off, epi=epi, avg_rows=max(512, Mt // E))
    for e in range(E):
        a, b = int(off[e]), int(off[e + 1])
        if a == b:
            continue
        r = (x[a:b].float() @ w[e].float().t()).to(bf)
        if epi:
            r = ref.silu_mul(ops.deinterleave_cols(r))
        close(y[a:b], r)


@pytest.mark.parametrize("counts,epi,N,K", [
    ([530, 498, 512, 470, 555, 505, 490, 528], 0, 4096, 14336),  # 19 slots x 16 = 304 tiles: 48 tail tiles in 4
    ([530, 498, 512, 470, 555, 505, 490, 528], 1, 28672, 4096),  # 2128 tiles: 80 tail tiles in 2 halves
    ([2000, 0, 0, 7, 0, 1500, 300, 281], 0, 4096, 14336),        # empty / tiny experts
    ([16, 17, 15, 16, 16, 18, 14, 16], 0, 4096, 14336),           # mid-size batch: split-K grouped (reduce)
    ([16, 16, 0, 30, 16, 10, 16, 24], 1, 28672, 4096),            # ... with the SiLU-mul epilogue in the reduce
    ([58, 54, 67, 83, 56, 59, 67, 68], 1, 28672, 4096),           # ~64 rows per expert: ping-pong from 56 (r5)
    ([120, 135, 160, 98, 140, 111, 130, 130], 0, 4096, 14336),    # ~128 rows: half-empty 256-row tiles
    ([257, 257, 257, 257, 257, 257, 257, 257], 1, 28672, 4096),   # decode-only spill: 1-row second tiles
])
def test_grouped_gemm_stream_k(gpu, counts, epi, N, K, grouped_balance):
    """Mixtral-size grouped GEMM with the stream-K tail planned ON DEVICE from the routed
    offsets (the host only knows the worst-case grid), three launches in a row, vs fp32
    per expert and vs the data-parallel grid."""
    torch.manual_seed(sum(counts) + N)
    ops._sk_reserve(torch.device(gpu))
    E = len(counts)
    off = torch.tensor([0] + list(np.cumsum(counts)), device=gpu, dtype=torch.int32)
    Mt = int(off[-1])
    x = torch.randn(Mt, K, device=gpu, dtype=bf)
    w = (0.02 * torch.randn(E, N, K, device=gpu)).to(bf)
    ys = [ops.grouped_gemm(x, w, off, epi=epi, avg_rows=Mt // E) for _ in range(3)]
    prev = torch.ops.mlop.gemm_sk_mode(-1)
    torch.ops.mlop.gemm_sk_mode(0)
    try:
        dp = ops.grouped_gemm(x, w, off, epi=epi, avg_rows=Mt // E)
    finally:
        torch.ops.mlop.gemm_sk_mode(prev)
    for e in range(E):
        a, b = int(off[e]), int(off[e + 1])
        if a == b:
            continue
        r = (x[a:b].float() @ w[e].float().t())
        if epi:
            r = ref.silu_mul(ops.deinterleave_cols(r.to(bf)))
        for y in ys + [dp]:
            close(y[a:b], r, atol=3e-2, rtol=3e-2)
    close(ys[0], ys[2], atol=0, rtol=0)


@pytest.mark.parametrize("counts", [[1, 0, 0, 0, 0, 0, 1, 0], [0, 3, 0, 2, 0, 0, 0, 3], [0, 0, 0, 0, 0, 0, 0, 1],
                                    [1, 1, 1, 1, 1, 1, 1, 1]])
@pytest.mark.parametrize("epi,N,K", [(1, 28672, 4096), (0, 4096, 14336), (1, 1024, 512), (0, 1024, 2048)])
def test_grouped_gemv_decode(gpu, counts, epi, N, K):
    """MoE decode (<= 8 routed rows): the grouped GEMV streams only the experts that got
    rows (grid = min(E, rows) expert slots), empty experts in between; vs fp32 per expert."""
    torch.manual_seed(sum(counts) * N)
    E = len(counts)
    off = torch.tensor([0] + list(np.cumsum(counts)), device=gpu, dtype=torch.int32)
    M = int(off[-1])
    x = torch.randn(M, K, device=gpu, dtype=bf)
    w = (0.03 * torch.randn(E, N, K, device=gpu)).to(bf)
    y = ops.grouped_gemm(x, w, off, epi=epi)
    for e in range(E):
        a, b = int(off[e]), int(off[e + 1])
        if a == b:
            continue
        r = (x[a:b].float() @ w[e].float().t()).to(bf)
        if epi:
            r = ref.silu_mul(ops.deinterleave_cols(r))
        close(y[a:b], r, atol=3e-2, rtol=3e-2)


@pytest.mark.parametrize("T,E,k,H", [(1, 8, 2, 4096), (4, 8, 2, 4096), (16, 8, 2, 1024), (7, 4, 1, 8192),
                                     (5, 64, 8, 2048)])
def test_moe_dispatch_small(gpu, T, E, k, H):
    """One-launch decode dispatch (router GEMV + route + sort + gather) against the
    separate router projection + moe_route + moe_permute, for the full and a partial
    (expert-parallel) local expert range."""
    torch.manual_seed(T * E)
    x = torch.randn(T, H, device=gpu, dtype=bf)
    wr = (0.05 * torch.randn(E, H, device=gpu)).to(bf)
    logits = (x.float() @ wr.float().t()).to(bf)
    p = torch.softmax(logits.float(), -1)
    for e0, nl in [(0, E), (E // 2, E - E // 2)]:
        topw, topi, xp, off, src, inv = ops.moe_dispatch_small(x, wr, k, e0, nl)
        w_ref, i_ref = ops.moe_route(logits, k)
        # bf16 logits tie often: compare the chosen probabilities, then the weights
        close(p.gather(1, topi.long()), p.gather(1, i_ref.long()), atol=1e-3, rtol=1e-3)
        close(topw, w_ref, atol=2e-3, rtol=2e-3)
        xp_r, off_r, _, inv_r = ops.moe_permute(x, topi, e0, nl)
        assert torch.equal(off.cpu(), off_r.cpu()) and torch.equal(inv.cpu(), inv_r.cpu())
        n = int(off[-1])
        close(xp[:n], xp_r[:n], atol=0, rtol=0)
        sel = torch.nonzero(inv >= 0).flatten()
        assert torch.equal(src[inv[sel].long()].cpu(), sel.to(torch.int32).cpu())


@pytest.mark.parametrize("T,E,k,H", [(1, 8, 2, 4096), (4, 8, 2, 4096), (16, 8, 2, 1024), (3, 8, 2, 8192)])
def test_moe_dispatch_small_prologue(gpu, T, E, k, H):
    """Dispatch with the residual add + RMSNorm prologue == add_rmsnorm, then dispatch."""
    torch.manual_seed(T + H)
    o = torch.randn(T, H, device=gpu, dtype=bf)
    res = torch.randn(T, H, device=gpu, dtype=bf)
    nw = (1 + 0.1 * torch.randn(H, device=gpu)).to(bf)
    wr = (0.05 * torch.randn(E, H, device=gpu)).to(bf)
    x_ref, res_ref = ref.add_rmsnorm(o, res, nw, 1e-5)
    r2 = res.clone()
    topw, topi, xp, off, src, inv = ops.moe_dispatch_small(o, wr, k, 0, E, pro=(o, r2, nw, 1e-5))
    close(r2, res_ref, atol=0, rtol=0)
    p = torch.softmax(x_ref.float() @ wr.float().t(), -1)
    w_ref, i_ref = ops.moe_route((x_ref.float() @ wr.float().t()).to(bf), k)
    close(p.gather(1, topi.long()), p.gather(1, i_ref.long()), atol=2e-3, rtol=2e-3)
    xp_r, off_r, _, inv_r = ops.moe_permute(x_ref, topi, 0, E)
    assert torch.equal(off.cpu(), off_r.cpu()) and torch.equal(inv.cpu(), inv_r.cpu())
    close(xp[:T * k], xp_r[:T * k], atol=2e-2, rtol=2e-2)


def _check_mid_layout(topi, off, arow, inv, T, k, e0, nl):
    """offsets = per-local-expert counts; every local slot s has a row in its expert's range
    whose token row is s // k; non-local slots are -1; rows are a permutation of [0, n)."""
    ti = topi.flatten().cpu().long() - e0
    local = (ti >= 0) & (ti < nl)
    counts = torch.bincount(ti[local], minlength=nl)
    assert torch.equal(off.cpu().long(), torch.cat([torch.zeros(1, dtype=torch.long), counts.cumsum(0)]))
    invc = inv.cpu().long()
    assert torch.all(invc[~local] == -1)
    rows = invc[local]
    assert torch.equal(rows.sort().values, torch.arange(int(off[-1])))
    lo, hi = off.cpu().long()[ti[local]], off.cpu().long()[ti[local] + 1]
    assert torch.all((rows >= lo) & (rows < hi))
    slots = torch.nonzero(local).flatten()
    assert torch.equal(arow.cpu().long()[rows], slots // k)


@pytest.fixture(params=[0, 2, 4, 8], ids=["tok_auto", "tok2", "tok4", "tok8"])
def mid_tok(request):
    """Tokens per workgroup of the mid MoE dispatch (moe_mid_tok): 0 = by T (default), 2, 4, 8."""
    prev = torch.ops.mlop.moe_mid_tok(-1)
    torch.ops.mlop.moe_mid_tok(request.param)
    yield request.param
    torch.ops.mlop.moe_mid_tok(prev)


@pytest.mark.parametrize("T,E,k,H", [(17, 8, 2, 4096), (64, 8, 2, 4096), (130, 8, 2, 1024), (1024, 8, 2, 4096), (5000, 8, 2, 4096),
                                     (40, 16, 4, 2048), (300, 8, 2, 8192)])
def test_moe_dispatch_mid(gpu, T, E, k, H, mid_tok):
    """Multi-workgroup dispatch (router GEMV + route per workgroup, last-workgroup sort, no
    gather) against the separate router projection + moe_route, for the full and a partial
    (expert-parallel) local expert range; twice in a row (the ticket resets itself)."""
    torch.manual_seed(T * E + H)
    x = torch.randn(T, H, device=gpu, dtype=bf)
    wr = (0.05 * torch.randn(E, H, device=gpu)).to(bf)
    logits = (x.float() @ wr.float().t()).to(bf)
    p = torch.softmax(logits.float(), -1)
    for e0, nl in [(0, E), (E // 2, E - E // 2), (0, E)]:
        topw, topi, xs, off, arow, inv = ops.moe_dispatch_mid(x, wr, k, e0, nl)
        assert xs.data_ptr() == x.data_ptr()  # no copy of the token rows
        w_ref, i_ref = ops.moe_route(logits, k)
        close(p.gather(1, topi.long()), p.gather(1, i_ref.long()), atol=1e-3, rtol=1e-3)
        close(topw, w_ref, atol=2e-3, rtol=2e-3)
        _check_mid_layout(topi, off, arow, inv, T, k, e0, nl)


@pytest.mark.parametrize("T,H", [(33, 4096), (200, 2048)])
def test_moe_dispatch_mid_prologue(gpu, T, H, mid_tok):
    """Mid dispatch with the residual add + RMSNorm prologue == add_rmsnorm, then route."""
    E, k = 8, 2
    torch.manual_seed(T + H)
    o = torch.randn(T, H, device=gpu, dtype=bf)
    res = torch.randn(T, H, device=gpu, dtype=bf)
    nw = (1 + 0.1 * torch.randn(H, device=gpu)).to(bf)
    wr = (0.05 * torch.randn(E, H, device=gpu)).to(bf)
    x_ref, res_ref = ref.add_rmsnorm(o, res, nw, 1e-5)
    r2 = res.clone()
    topw, topi, xs, off, arow, inv = ops.moe_dispatch_mid(o, wr, k, 0, E, pro=(o, r2, nw, 1e-5))
    close(r2, res_ref, atol=0, rtol=0)
    close(xs, x_ref, atol=2e-2, rtol=2e-2)
    p = torch.softmax(x_ref.float() @ wr.float().t(), -1)
    w_ref, i_ref = ops.moe_route((x_ref.float() @ wr.float().t()).to(bf), k)
    close(p.gather(1, topi.long()), p.gather(1, i_ref.long()), atol=2e-3, rtol=2e-3)
    _check_mid_layout(topi, off, arow, inv, T, k, 0, E)


@pytest.mark.parametrize("T,H,I", [(24, 1024, 512), (64, 4096, 1024), (300, 1024, 512)])
def test_moe_block_mid_dispatch_matches_fp32(gpu, T, H, I):
    """The whole single-rank MoE block through the mid dispatch (grouped GEMMs reading x via
    arow, combine + add + RMSNorm) against the fp32 reference MoE on the same routing."""
    from mlopamd.parallel import moe as moe_mod

    E, k = 8, 2
    torch.manual_seed(T + I)
    x = torch.randn(T, H, device=gpu, dtype=bf)
    wr = (0.05 * torch.randn(E, H, device=gpu)).to(bf)
    w13 = (0.03 * torch.randn(E, 2 * I, H, device=gpu)).to(bf)
    w2 = (0.03 * torch.randn(E, H, I, device=gpu)).to(bf)
    res = torch.randn(T, H, device=gpu, dtype=bf)
    nw = (1 + 0.1 * torch.randn(H, device=gpu)).to(bf)
    mid = ops.moe_dispatch_mid(x, wr, k, 0, E)
    assert mid is not None
    topw, topi = mid[0], mid[1]
    r2 = res.clone()
    out = moe_mod.moe_forward_add_norm(x, wr, w13, w2, k, 0, E, r2, nw, 1e-5)
    # fp32 oracle on the kernel's own routing (bf16 logits may tie differently in torch)
    xf = x.float()
    y = torch.zeros(T, H, device=gpu)
    for t in range(T):
        for j in range(k):
            e = int(topi[t, j])
            gu = xf[t] @ w13[e].float().t()  # w13 rows gate / up interleaved in groups of 16
            h = ref.silu_mul(ops.deinterleave_cols(gu.to(bf).view(1, -1))).float().view(-1)
            y[t] += topw[t, j] * (h.to(bf).float() @ w2[e].float().t())
    exp_out, exp_res = ref.add_rmsnorm(y.to(bf), res, nw, 1e-5)
    close(r2, exp_res, atol=3e-2, rtol=3e-2)
    close(out, exp_out, atol=5e-2, rtol=5e-2)


@pytest.mark.parametrize("T,k,H", [(1, 2, 4096), (9, 2, 4096), (3, 1, 8192), (16, 8, 2048)])
def test_moe_combine_add_rmsnorm(gpu, T, k, H):
    torch.manual_seed(H + T)
    rows = T * k
    y = torch.randn(rows, H, device=gpu, dtype=bf)
    inv = torch.randperm(rows, device=gpu).to(torch.int32)
    inv[0] = -1  # a slot routed to another rank's expert
    topw = torch.rand(T, k, device=gpu)
    res = torch.randn(T, H, device=gpu, dtype=bf)
    nw = (1 + 0.1 * torch.randn(H, device=gpu)).to(bf)
    exp_out, exp_res = ref.add_rmsnorm(ops.moe_combine(y, inv, topw), res, nw, 1e-5)
    r2 = res.clone()
    out = ops.moe_combine_add_rmsnorm(y, inv, topw, r2, nw, 1e-5)
    close(r2, exp_res, atol=0, rtol=0)
    close(out, exp_out, atol=2e-2, rtol=2e-2)


@pytest.mark.parametrize("T,E,k,H,I", [(1, 8, 2, 4096, 1024), (3, 8, 2, 4096, 14336), (77, 8, 2, 1024, 512),
                                       (512, 8, 2, 512, 256), (300, 4, 1, 256, 256)])
def test_moe_pipeline(gpu, T, E, k, H, I):
    torch.manual_seed(T)
    x = torch.randn(T, H, device=gpu, dtype=bf)
    logits = torch.randn(T, E, device=gpu, dtype=bf)
    w, idx = ops.moe_route(logits, k)
    w_ref, idx_ref = ref.moe_route(logits, k)
    # bf16 router logits tie often: compare the chosen probabilities, not tie-broken ids
    p = torch.softmax(logits.float(), -1)
    torch.testing.assert_close(p.gather(1, idx.long()).cpu(), p.gather(1, idx_ref.long()).cpu())
    close(w, w_ref, atol=1e-5, rtol=1e-4)
    w13 = (0.05 * torch.randn(E, 2 * I, H, device=gpu)).to(bf)
    w2 = (0.05 * torch.randn(E, H, I, device=gpu)).to(bf)
    for e0, nl in [(0, E), (E // 2, E - E // 2)]:
        xp, off, src, inv = ops.moe_permute(x, idx, e0, nl)
        xp_r, off_r, src_r, inv_r = ref.moe_permute(x, idx, e0, nl)
        assert torch.equal(off.cpu(), off_r.cpu())
        n = int(off[-1])
        # same rows per expert (order inside an expert may differ): compare via inv
        assert torch.equal((inv >= 0).cpu(), (inv_r >= 0).cpu())
        close(xp[inv[inv >= 0].long()], x[(torch.nonzero(inv >= 0).flatten() // k)], atol=0, rtol=0)
        a = ops.grouped_gemm(xp, w13[e0:e0 + nl], off, epi=ops.EPI_SILU_MUL)
        y = ops.grouped_gemm(a, w2[e0:e0 + nl], off)
        out = ops.moe_combine(y, inv, w)
        # reference: dense per-slot expert compute
        exp = torch.zeros(T, H, device=gpu)
        for t in range(T):
            for j in range(k):
                e = int(idx[t, j])
                if not (e0 <= e < e0 + nl):
                    continue
                gu = (x[t].float() @ ops.deinterleave_rows(w13[e]).float().t()).to(bf)
                h = ref.silu_mul(gu[None])[0].float() @ w2[e].float().t()
                exp[t] += w[t, j] * h.to(bf).float()
        # bf16 rounding noise scales with the output magnitude (large I: |out| ~ 20)
        close(out, exp, atol=3e-2 + 3e-3 * float(exp.abs().max()), rtol=3e-2)
        assert n == int(((idx >= e0) & (idx < e0 + nl)).sum())


@pytest.mark.parametrize("M", [16, 64, 200, 600])
def test_nt_weight_policy_bit_identical(gpu, M):
    """The non-temporal weight stream (gemm_small_nt: one-m-tile dense tiles, grouped small
    tiles, grouped ping-pong) changes the cache policy only: outputs are bit-identical to the
    default policy, dense and grouped."""
    torch.manual_seed(M)
    ops._sk_reserve(torch.device(gpu))
    x = torch.randn(M, 4096, device=gpu, dtype=bf)
    w = (0.02 * torch.randn(6144, 4096, device=gpu)).to(bf)
    E = 8
    counts = [M // E + (1 if e < M % E else 0) for e in range(E)]
    off = torch.tensor([0] + list(np.cumsum(counts)), device=gpu, dtype=torch.int32)
    we = (0.02 * torch.randn(E, 1024, 4096, device=gpu)).to(bf)
    prev_b = ops.GEMM_BACKEND
    prev = torch.ops.mlop.gemm_small_nt(-1)
    outs = {}
    try:
        ops.GEMM_BACKEND = "mlop"
        for nt in (0, 7):
            torch.ops.mlop.gemm_small_nt(nt)
            outs[nt] = (ops.gemm(x, w), ops.gemm(x, w[:4096], epi=ops.EPI_SILU_MUL),
                        ops.grouped_gemm(x, we, off, epi=0, avg_rows=max(1, M // E)))
    finally:
        torch.ops.mlop.gemm_small_nt(prev)
        ops.GEMM_BACKEND = prev_b
    for a, b in zip(outs[0], outs[7]):
        assert torch.equal(a, b)
    close(outs[7][0], (x.float() @ w.float().t()).to(bf))


@pytest.mark.parametrize("case", ["decode", "split"])
def test_attention_kv_policy_bit_identical(gpu, case):
    """Non-temporal K / V page loads and output stores in the decode kernel (attn_kv_nt):
    bit-identical output."""
    torch.manual_seed(3)
    np.random.seed(3)
    Hq, Hkv = 32, 8
    # >= 8 query tiles: the policy applies from 8 (below, the default policy always)
    ctx = [300, 1000, 17, 64, 900, 33, 512, 700] if case == "decode" else [3000, 2500] * 4
    NB = sum((c + 15) // 16 for c in ctx) + 8
    kc = torch.randn(NB, Hkv, 16, 128, device=gpu, dtype=bf)
    vc = torch.randn(NB, Hkv, 16, 128, device=gpu, dtype=bf)
    kw = dict(part_tokens=512, nparts=6) if case == "split" else {}
    m, T = make_meta(gpu, [1] * len(ctx), ctx, Hkv, Hq // Hkv, NB, **kw)
    q = torch.randn(T, Hq, 128, device=gpu, dtype=bf)
    prev = torch.ops.mlop.attn_kv_nt(-1)
    try:
        torch.ops.mlop.attn_kv_nt(0)
        a = ops.paged_attention(q, kc, vc, m).clone()
        torch.ops.mlop.attn_kv_nt(3)
        b = ops.paged_attention(q, kc, vc, m).clone()
    finally:
        torch.ops.mlop.attn_kv_nt(prev)
    assert torch.equal(a, b)
    close(b, ref.paged_attention(q, kc, vc, m))



@pytest.fixture
def ws_on():
    """The weight-streaming MFMA kernel is off in serving (gemm_ws_max_m = 0): on for the test."""
    prev = torch.ops.mlop.gemm_ws_max_m(-1)
    torch.ops.mlop.gemm_ws_max_m(64)
    yield
    torch.ops.mlop.gemm_ws_max_m(prev)
    torch.ops.mlop.gemm_ws_plan(0, 0, 1)


@pytest.mark.parametrize("plan", [(0, 0, 1), (4, 4, 0), (2, 8, 1)], ids=["default", "rb4u4c", "rb2u8nt"])
@pytest.mark.parametrize("M", [5, 16, 17, 33, 64])
@pytest.mark.parametrize("N,K,epi", [(1024, 4096, 0), (2048, 4096, 1), (512, 14336, 0), (4096, 1024, 0)])
def test_gemm_ws_vs_fp32(gpu, ws_on, plan, M, N, K, epi):
    """K2 at 5-64 rows, the weight-streaming MFMA kernel (gemm_ws.hip): plain and SiLU-mul
    (16-interleaved gate / up rows) against the fp32 product; rows past M are never written."""
    from mlopamd import ops

    torch.manual_seed(M * 7 + N)
    torch.ops.mlop.gemm_ws_plan(*plan)
    a = torch.randn(M, K, device=gpu, dtype=torch.bfloat16)
    w = (0.02 * torch.randn(N, K, device=gpu)).to(torch.bfloat16)
    out = torch.full((M + 3, N // 2 if epi else N), 7.0, device=gpu, dtype=torch.bfloat16)
    assert torch.ops.mlop.gemm_ws(out[:M], a, w, epi, False, 0.0)
    exp = a.float() @ w.float().t()
    if epi:
        exp = ops.reference.silu_mul(ops.deinterleave_cols(exp.to(torch.bfloat16))).float()
    torch.testing.assert_close(out[:M].float(), exp, atol=2e-2 * exp.abs().max().item() / 4 + 1e-2, rtol=2e-2)
    assert bool((out[M:] == 7.0).all())
    # deterministic relaunch
    out2 = torch.empty_like(out[:M])
    torch.ops.mlop.gemm_ws(out2, a, w, epi, False, 0.0)
    assert torch.equal(out2, out[:M])
