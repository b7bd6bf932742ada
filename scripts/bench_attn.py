"""Prefill attention microbench (Llama-3-8B heads: 32 q / 8 kv, D=128): the K7
flash-prefill kernel vs the decode-tile kernel on the same ragged paged cache,
vs torch SDPA (causal, contiguous, GQA expanded).  Causal FLOPs = 2*2*L^2/2*D*Hq."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
from mlopamd import ops  # noqa: E402
from test_kernels_gpu import make_meta  # noqa: E402

ops.load()
dev = torch.device("cuda")
bf = torch.bfloat16
Hq, Hkv, D = 32, 8, 128


def timeit(fn, iters=10):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


for L, nseq in ((512, 16), (2048, 4), (8192, 1)):
    np.random.seed(0)
    NB = nseq * ((L + 15) // 16) + 8
    kc = torch.randn(NB, Hkv, 16, D, device=dev, dtype=bf)
    vc = torch.randn(NB, Hkv, D, 16, device=dev, dtype=bf)
    mf, T = make_meta(dev, [L] * nseq, [L] * nseq, Hkv, Hq // Hkv, NB, flash_min_q=17)
    md, _ = make_meta(dev, [L] * nseq, [L] * nseq, Hkv, Hq // Hkv, NB)
    q = torch.randn(T, Hq, D, device=dev, dtype=bf)
    t_flash = timeit(lambda: ops.paged_attention(q, kc, vc, mf))
    t_tile = timeit(lambda: ops.paged_attention(q, kc, vc, md), iters=3)
    qs = torch.randn(nseq, Hq, L, D, device=dev, dtype=bf)
    ks = torch.randn(nseq, Hq, L, D, device=dev, dtype=bf)
    vs = torch.randn(nseq, Hq, L, D, device=dev, dtype=bf)
    t_sdpa = timeit(lambda: torch.nn.functional.scaled_dot_product_attention(qs, ks, vs, is_causal=True))
    fl = nseq * 2 * 2 * L * L / 2 * D * Hq
    print(json.dumps(dict(L=L, nseq=nseq, flash_us=round(t_flash, 1), tile_us=round(t_tile, 1),
                          sdpa_us=round(t_sdpa, 1), flash_tflops=round(fl / t_flash / 1e6, 1),
                          sdpa_tflops=round(fl / t_sdpa / 1e6, 1))), flush=True)
