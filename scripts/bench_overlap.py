"""Nano-batch overlap feasibility: does running two independent halves of a mixed
step on two HIP streams (one half's HBM-bound decode attention next to the other
half's MFMA-bound projections) beat the single big batch run serially?

Per layer (Llama-3-8B shapes): qkv GEMM, decode paged attention, o GEMM,
gate_up GEMM (+SiLU-mul), down GEMM.  'serial' = one batch of M rows with
B decode sequences; 'nano' = two batches of M/2 rows and B/2 sequences issued
layer-interleaved on two streams.  Reports ms per 32-layer forward."""
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
H, I, Hq, Hkv, D = 4096, 14336, 32, 8, 128
LAYERS = int(os.environ.get("LAYERS", 32))
M_TOTAL = int(os.environ.get("M", 3840))
B_TOTAL = int(os.environ.get("B", 2048))
CTX = int(os.environ.get("CTX", 387))

w_qkv = (0.02 * torch.randn((Hq + 2 * Hkv) * D, H, device=dev)).to(bf)
w_o = (0.02 * torch.randn(H, Hq * D, device=dev)).to(bf)
w_gu = (0.02 * torch.randn(2 * I, H, device=dev)).to(bf)
w_dn = (0.02 * torch.randn(H, I, device=dev)).to(bf)


class Half:
    def __init__(self, M, B, seed):
        np.random.seed(seed)
        ctx = np.random.randint(CTX // 2, CTX * 3 // 2 + 1, size=B).tolist()
        NB = sum((c + 15) // 16 for c in ctx) + 8
        self.kc = torch.randn(NB, Hkv, 16, D, device=dev, dtype=bf)
        self.vc = torch.randn(NB, Hkv, 16, D, device=dev, dtype=bf)
        self.meta, T = make_meta(dev, [1] * B, ctx, Hkv, Hq // Hkv, NB)
        self.q = torch.randn(T, Hq, D, device=dev, dtype=bf)
        self.x = torch.randn(M, H, device=dev, dtype=bf)
        self.M, self.B = M, B

    def layer(self):
        ops.gemm(self.x, w_qkv)
        a = ops.paged_attention(self.q, self.kc, self.vc, self.meta)
        ops.gemm(self.x, w_o)  # o-proj input shape stand-in (same M x 4096)
        h = ops.gemm(self.x, w_gu, epi=ops.EPI_SILU_MUL)
        ops.gemm(h, w_dn)
        return a


def timeit(fn, iters=3):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


full = Half(M_TOTAL, B_TOTAL, 0)
ha, hb = Half(M_TOTAL // 2, B_TOTAL // 2, 1), Half(M_TOTAL // 2, B_TOTAL // 2, 2)
sa, sb = torch.cuda.Stream(), torch.cuda.Stream()


def serial():
    for _ in range(LAYERS):
        full.layer()


def halves_serial():
    for _ in range(LAYERS):
        ha.layer()
        hb.layer()


def nano():
    cur = torch.cuda.current_stream()
    sa.wait_stream(cur)
    sb.wait_stream(cur)
    for _ in range(LAYERS):
        with torch.cuda.stream(sa):
            ha.layer()
        with torch.cuda.stream(sb):
            hb.layer()
    cur.wait_stream(sa)
    cur.wait_stream(sb)


def attn_only():
    for _ in range(LAYERS):
        ops.paged_attention(full.q, full.kc, full.vc, full.meta)


def gemm_only():
    for _ in range(LAYERS):
        ops.gemm(full.x, w_qkv)
        ops.gemm(full.x, w_o)
        h = ops.gemm(full.x, w_gu, epi=ops.EPI_SILU_MUL)
        ops.gemm(h, w_dn)


res = {}
for _ in range(2):
    for name, fn in (("serial", serial), ("halves_serial", halves_serial), ("nano_2stream", nano),
                     ("attn_only", attn_only), ("gemm_only", gemm_only)):
        t = timeit(fn)
        res[name] = min(res.get(name, 1e9), t)
print(json.dumps(dict(M=M_TOTAL, B=B_TOTAL, ctx=CTX, layers=LAYERS, **{k: round(v, 2) for k, v in res.items()},
                      gemm_backends=ops.gemm_choices())), flush=True)


# ---------------------------------------------------------------------------------------
# CU-partitioned pipeline (ATTN_CUS > 0): GEMMs on a stream masked to the other CUs,
# decode attention on a stream masked to ATTN_CUS CUs (the same number in every XCD whether
# the CU ids count XCD-major (i // 32) or round-robin (i % 8)),
# two half batches interleaved so one half's attention runs beside the other half's MLP:
#   G: qkvA(l) mlpB(l-1) qkvB(l) mlpA(l) ...      T: attnA(l) attnB(l) ...
def cu_mask_stream(cus):
    import ctypes

    lib = ctypes.CDLL(os.path.join(os.path.dirname(torch.__file__), "lib", "libamdhip64.so"))
    n = torch.cuda.get_device_properties(0).multi_processor_count
    words = [0] * ((n + 31) // 32)
    for i in cus:
        words[i // 32] |= 1 << (i % 32)
    arr = (ctypes.c_uint32 * len(words))(*words)
    h = ctypes.c_void_p()
    err = lib.hipExtStreamCreateWithCUMask(ctypes.byref(h), ctypes.c_uint32(len(words)), arr)
    assert err == 0, f"hipExtStreamCreateWithCUMask: {err}"
    return torch.cuda.ExternalStream(h.value)


ATTN_CUS = int(os.environ.get("ATTN_CUS", 0))
if ATTN_CUS:
    n = torch.cuda.get_device_properties(0).multi_processor_count
    per = ATTN_CUS // 8  # attention CUs per 32-CU block, spread over the mod-8 classes too
    # balanced pick: in 32-CU block b take CUs b*32 + 4*k + (b % 4), k < per
    attn_set = [b * 32 + 4 * k + (b % 4) for b in range(n // 32) for k in range(per)]
    gemm_set = [i for i in range(n) if i not in set(attn_set)]
    G, Tst = cu_mask_stream(gemm_set), cu_mask_stream(attn_set)

    def mlp(h):
        ops.gemm(h.x, w_o)
        a = ops.gemm(h.x, w_gu, epi=ops.EPI_SILU_MUL)
        ops.gemm(a, w_dn)

    def pipelined():
        cur = torch.cuda.current_stream()
        G.wait_stream(cur)
        Tst.wait_stream(cur)
        ev = {}
        for l in range(LAYERS):
            for h, tag in ((ha, "A"), (hb, "B")):
                with torch.cuda.stream(G):
                    ops.gemm(h.x, w_qkv)
                    e = torch.cuda.Event()
                    e.record(G)
                with torch.cuda.stream(Tst):
                    Tst.wait_event(e)
                    ops.paged_attention(h.q, h.kc, h.vc, h.meta)
                    ea = torch.cuda.Event()
                    ea.record(Tst)
                # the OTHER half's MLP of the previous step runs now on G
                other, otag = (hb, "B") if tag == "A" else (ha, "A")
                key = "pending" + otag
                if key in ev:
                    with torch.cuda.stream(G):
                        G.wait_event(ev.pop(key))
                        mlp(other)
                ev["pending" + tag] = ea
        for tag, h in (("A", ha), ("B", hb)):
            if "pending" + tag in ev:
                with torch.cuda.stream(G):
                    G.wait_event(ev.pop("pending" + tag))
                    mlp(h)
        cur.wait_stream(G)
        cur.wait_stream(Tst)

    def attn_masked():
        cur = torch.cuda.current_stream()
        Tst.wait_stream(cur)
        with torch.cuda.stream(Tst):
            for _ in range(LAYERS):
                ops.paged_attention(ha.q, ha.kc, ha.vc, ha.meta)
        cur.wait_stream(Tst)

    def gemm_masked():
        cur = torch.cuda.current_stream()
        G.wait_stream(cur)
        with torch.cuda.stream(G):
            for _ in range(LAYERS):
                ops.gemm(ha.x, w_qkv)
                mlp(ha)
        cur.wait_stream(G)

    r2 = {}
    for _ in range(2):
        for name, fn in (("pipelined", pipelined), ("halves_serial", halves_serial),
                         ("half_attn_on_attn_cus", attn_masked), ("half_gemms_on_gemm_cus", gemm_masked)):
            t = timeit(fn)
            r2[name] = min(r2.get(name, 1e9), t)
    print(json.dumps(dict(M=M_TOTAL, B=B_TOTAL, ctx=CTX, layers=LAYERS, attn_cus=len(attn_set),
                          **{k: round(v, 2) for k, v in r2.items()})), flush=True)
