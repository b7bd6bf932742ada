"""Generator of ``csrc/gemm_w4_asm.h``: the hand-scheduled K-loop of the four-wave
256 x 256 bf16 GEMM (``csrc/gemm_w4.hip``) as one inline-asm statement.

Why asm: the loop's value is its instruction ORDER -- every MFMA followed by at most one
LDS read or LDS-DMA issue, barriers placed between MFMAs so the matrix pipe keeps running
while a wave waits, counted ``lgkmcnt`` per fragment and ``vmcnt`` per tile.  hipcc
re-orders such a body (a compiler-scheduled four-wave version of the same tiling measured
126-137 us at 4096^3 vs 103 us for the two-group ping-pong kernel,
``profiles/r03_gemm_fourwave.md``).  With one wave per SIMD the only latency hiding is
the interleave itself, so it is written out here instruction by instruction.

Geometry (one workgroup = 4 waves = one 256 x 256 output tile, BK = 64):
  * wave w = (wm, wn) = (w >> 1, w & 1) owns rows wm*128 .. +127, cols wn*128 .. +127:
    8 x 8 accumulators of v_mfma_f32_16x16x32_bf16 = 256 AGPRs (a[4(8i+j) .. +3]), computed
    transposed (B fragment as the MFMA's A operand): acc(i, j)[r] of lane l is
    C[16i + (l & 15)][16j + 4(l >> 4) + r];
  * LDS: two 64 KiB buffers; buffer b = A rows 0-255 (32 KiB) then B rows 0-255, each row
    128 B (64 bf16 of K), 16-B chunk c of row r at slot c ^ ((r >> 1) & 7) (the swizzle rides
    in the DMA SOURCE address; the LDS image is lane-linear per 1 KiB piece);
  * per K-tile a wave issues 16 LDS-DMA pieces (buffer_load_dwordx4 ... lds; piece
    p = w + 4i, i = 0..15: i < 8 A rows 8p.., else B rows 8(p - 32)..) and 32 ds_read_b128
    (A and B fragments for both 32-deep K halves) against 128 MFMAs.

Schedule of iteration t (MFMA slot m = 0..127; H0 = k-half 0 of tile t, H1 = k-half 1):
  m  1..31   ds_read k-half-1 fragments of tile t (FB1[0..7], FA1[0..7]) from buffer t&1
  m  38      lgkmcnt(0) + s_barrier (B1): every wave is done reading buffer t&1
  m 40..100  16 LDS-DMA pieces of tile t+2 into buffer t&1 (one per 4 MFMAs)
  m  102     vmcnt(16) + s_barrier (B2): tile t+1 (issued one iteration ago) has landed
  m 103..127 ds_read k-half-0 fragments of tile t+1 (FB0, FA0) from buffer (t+1)&1
MFMA order: H0 = (i, j) row-major over FA0[i] x FB0[j]; H1 = the same over FA1 x FB1.
lgkmcnt waits are derived here from the in-order LDS return queue (each MFMA waits only
for the fragments it reads).  The last two iterations are peeled: t = nk-2 issues no DMA
(B2 waits vmcnt(0)), t = nk-1 issues neither DMA nor next-tile reads.

Hazards handled in the text (hipcc pads nothing inside an asm statement):
  * s_mov/s_add m0 -> LDS-DMA: at least one MFMA between them;
  * fragment registers are rewritten >= 8 MFMAs after their last MFMA reader;
  * v_accvgpr_write (zeroing) -> first MFMA: the prologue's barrier + reads lie between;
  * last MFMA -> v_accvgpr_read (readout statements): 3 x s_nop 7 at the end.

Half-height variant (BM = 128, round 5): the same schedule shape over 64 MFMAs per K-tile --
each wave owns 64 x 128 outputs (4 x 8 accumulators, 128 AGPRs), the A operand is 128 rows
(4 fragments per k-half, 4 of the 12 LDS-DMA pieces per wave), so a grid has twice the tiles
(QKV at M = 4088: 768 tiles = 3 whole rounds of the 256 CUs instead of 1.5; O at 1536-2560 rows
one full round instead of K-half tails).  Slots: rd1 at 1..12, B1 at 20 (8 MFMAs of slack for
the reads' return), 12 DMAs at 21..43, B2 at 45, rd0 at 46..57 (6 MFMAs of slack before the next
K-tile's first MFMA); the fragment-reuse distance (>= 8 MFMAs) holds as in the full tile.

Run ``python -m mlopamd.ops.gen_gemm_w4`` to regenerate the header (committed; the build
does not run Python).
"""
from __future__ import annotations

from pathlib import Path

OUT = Path(__file__).resolve().parent / "csrc" / "gemm_w4_asm.h"

NFB = 8           # B fragments per k-half (8 x 16 columns: the wave's 128 columns)


class Sched:
    """Slot placement of one K-tile iteration (slot m = before MFMA m) for a tile of ``bm`` rows:
    ``nfa`` = bm / 32 A fragments per wave and k-half, ``na`` = bm / 32 A pieces of the ``npc``
    LDS-DMA pieces per wave, ``nmma`` MFMAs per K-tile."""

    def __init__(self, rd1, b1, dma, b2, rd0, toggle1=60, pol_a="", pol_b="", bm=256):
        self.rd1, self.b1, self.dma, self.b2, self.rd0, self.toggle1 = rd1, b1, dma, b2, rd0, toggle1
        self.pol = {"srdA": pol_a, "srdB": pol_b}  # cache-policy bits of each operand's LDS-DMA
        self.bm = bm
        self.nfa = bm // 32
        self.na = bm // 32
        self.npc = self.na + 8
        self.nmma = 2 * self.nfa * NFB
        self.loopctl = self.nmma - 1
        nrd = NFB + self.nfa
        assert len(rd1) == nrd and len(rd0) == nrd and len(dma) == self.npc
        assert max(rd1) < b1 < min(dma) and b2 < min(rd0) and max(rd0) <= self.nmma - 1 and toggle1 > max(rd1)
        self.dma_before_b2 = sum(1 for m in dma if m < b2)


# All 16 DMAs between the barriers (one per 4 MFMAs), next-tile reads packed at the end.
# Measured and dropped (profiles/r03_gemm_w4.md): B2 at MFMA 86 with one DMA per 3 MFMAs, a
# hipBLASLt-like 8 + 8 DMA split around B2 at the half boundary (both within 1 %), and
# non-temporal weight / activation DMAs (2-8 % slower).
SCHEDS = [Sched(rd1=[1 + 2 * k for k in range(16)], b1=38, dma=[40 + 4 * k for k in range(16)], b2=102,
                rd0=[103 + round(k * 24 / 15) for k in range(16)])]
# the half-height tile (BM = 128): 64 MFMAs, 12 fragment reads per k-half, 12 DMA pieces
SCHED_H = Sched(rd1=[1 + k for k in range(12)], b1=20, dma=[21 + 2 * k for k in range(12)], b2=45,
                rd0=[46 + k for k in range(12)], toggle1=19, bm=128)


def frag(name, i):
    return f"%[{name}{i}]"


def mfma(q, a, b, zero_c=False):
    # B fragment as the MFMA's A operand: the accumulator holds C^T, so lane l owns C row
    # (l & 15) of the fragment and FOUR consecutive columns 4(l >> 4) .. +3 -- one 8-byte
    # store per accumulator in the epilogue instead of four 2-byte ones
    c = "0" if zero_c else f"a[{4 * q}:{4 * q + 3}]"
    return f"v_mfma_f32_16x16x32_bf16 a[{4 * q}:{4 * q + 3}], {b}, {a}, {c}"


class Stream:
    """Emits instructions and tracks the in-order LDS-read return queue."""

    def __init__(self):
        self.lines: list[str] = []
        self.queue: list[str] = []   # outstanding ds_read destinations, issue order

    def emit(self, s):
        self.lines.append(s)

    def read(self, dst, addr, off):
        self.emit(f"ds_read_b128 {frag(*dst)}, %[{addr}] offset:{off}")
        self.queue.append(dst)

    def need(self, *dsts):
        """Wait until every fragment in dsts has returned."""
        pos = [self.queue.index(d) for d in dsts if d in self.queue]
        if not pos:
            return
        p = max(pos)
        cnt = len(self.queue) - 1 - p
        self.emit(f"s_waitcnt lgkmcnt({min(cnt, 15)})")
        # lgkmcnt(c) retires everything but the newest c ops (and at least the first p+1)
        keep = min(cnt, 15)
        self.queue = self.queue[len(self.queue) - keep:] if keep else []

    def drain(self):
        self.emit("s_waitcnt lgkmcnt(0)")
        self.queue = []


def reads_k1(sc: Sched):
    """ds_reads of the k-half-1 fragments (FB1 then FA1) of the current tile."""
    return [(("fb1_", j), "rB1", j * 2048) for j in range(NFB)] + [(("fa1_", i), "rA1", i * 2048) for i in range(sc.nfa)]


def reads_k0(sc: Sched):
    return [(("fb0_", j), "rB0", j * 2048) for j in range(NFB)] + [(("fa0_", i), "rA0", i * 2048) for i in range(sc.nfa)]


def body(s: Stream, sc: Sched, kind: str, first: bool = False):
    """One K-tile iteration. kind: steady (DMA t+2, reads t+1), nodma (reads t+1), last.
    first: the tile's K-tile 0 -- the H0 MFMAs start the accumulators from 0 (no zeroing pass)."""
    dma = kind == "steady"
    nxt = kind != "last"
    NM = sc.nmma
    slots: dict[int, list] = {m: [] for m in range(NM + 1)}
    for m, op in zip(sc.rd1, reads_k1(sc)):
        slots[m].append(("read", op))
    if dma:
        slots[sc.b1].append(("b1",))
        slots[sc.dma[0] - 1].append(("emit", "s_mov_b32 m0, %[dbase]"))
        for k, m in enumerate(sc.dma):
            srd = "srdA" if k < sc.na else "srdB"
            slots[m].append(("emit", f"buffer_load_dwordx4 %[vo{k}], %[{srd}], %[koff] offen{sc.pol[srd]} lds"))
            if k < sc.npc - 1:
                slots[m].append(("emit", "s_add_u32 m0, m0, 0x1000"))
        slots[sc.dma[-1] + 1].append(("emit", "s_add_u32 %[koff], %[koff], 0x80"))
        slots[sc.dma[-1] + 1].append(("emit", "s_xor_b32 %[dbase], %[dbase], 0x10000"))
    slots[sc.toggle1].append(("emit", "v_xor_b32_e32 %[rA1], 0x10000, %[rA1]"))
    slots[sc.toggle1].append(("emit", "v_xor_b32_e32 %[rB1], 0x10000, %[rB1]"))
    if nxt:
        slots[sc.b2].append(("b2", sc.dma_before_b2 if dma else 0))
        slots[sc.b2].append(("emit", "v_xor_b32_e32 %[rA0], 0x10000, %[rA0]"))
        slots[sc.b2].append(("emit", "v_xor_b32_e32 %[rB0], 0x10000, %[rB0]"))
        for m, op in zip(sc.rd0, reads_k0(sc)):
            slots[m].append(("read", op))
    if kind == "steady" and not first:
        slots[sc.loopctl].append(("emit", "s_sub_u32 %[iter], %[iter], 1"))
        slots[sc.loopctl].append(("emit", "s_cmp_lg_u32 %[iter], 0"))
    for m in range(NM + 1):
        for op in slots[m]:
            if op[0] == "read":
                dst, addr, off = op[1]
                s.read(dst, addr, off)
            elif op[0] == "emit":
                s.emit(op[1])
            elif op[0] == "b1":
                s.drain()
                s.emit("s_barrier")
            elif op[0] == "b2":
                s.emit(f"s_waitcnt vmcnt({op[1]})")
                s.emit("s_barrier")
        if m == NM:
            break
        h, mm = divmod(m, NM // 2)
        i, j = divmod(mm, NFB)
        a, b = (("fa0_", i), ("fb0_", j)) if h == 0 else (("fa1_", i), ("fb1_", j))
        s.need(a, b)
        s.emit(mfma(NFB * i + j, frag(*a), frag(*b), zero_c=first and h == 0))


def suffix(q, q0):
    """lgkmcnt(N) = 'all but the N newest LDS ops returned': waits derived for the queue q0
    stay correct for any actual queue that is a suffix of q0 (older entries already retired)."""
    return q0[len(q0) - len(q):] == q


def issue_two(s: Stream, vo: str, sc: Sched):
    """LDS-DMA of a tile's K-tiles 0 and 1 into buffers 0 and 1 (per-lane offsets %[{vo}k])."""
    for t in range(2):
        s.emit("s_mov_b32 m0, %[dbase]" if t == 0 else "s_xor_b32 m0, %[dbase], 0x10000")
        s.emit("s_nop 0")
        for k in range(sc.npc):
            srd = "srdA" if k < sc.na else "srdB"
            soff = "0" if t == 0 else "%[k128]"
            s.emit(f"buffer_load_dwordx4 %[{vo}{k}], %[{srd}], {soff} offen{sc.pol[srd]} lds")
            if k < sc.npc - 1:
                s.emit("s_add_u32 m0, m0, 0x1000")
                s.emit("s_nop 0")


def kloop(n_stores: int, sc: Sched) -> list[str]:
    """One output tile.  Entry: %[first] != 0 -> issue this tile's K-tiles 0 / 1 here; else
    the previous tile's statement issued them, followed by exactly n_stores epilogue store
    instructions (vmcnt counts both in issue order).  Exit: %[has_next] != 0 -> K-tiles 0 / 1
    of the next tile (offsets %[vn*]) are issued into the freed buffers before returning, so
    their latency hides behind this tile's epilogue."""
    s = Stream()
    # s_nop 4: the descriptor / m0 SGPRs may come straight from v_readfirstlane
    s.emit("s_nop 4")
    s.emit("s_mov_b32 %[m0save], m0")
    s.emit("s_cmp_eq_u32 %[first], 0")
    s.emit("s_cbranch_scc1 L_w4_pref_%=")
    issue_two(s, "vo", sc)
    s.emit(f"s_waitcnt vmcnt({sc.npc})")
    s.emit("s_branch L_w4_go_%=")
    s.emit("L_w4_pref_%=:")
    assert sc.npc + n_stores <= 63
    s.emit(f"s_waitcnt vmcnt({sc.npc + n_stores})")
    s.emit("L_w4_go_%=:")
    s.emit("s_barrier")
    for dst, addr, off in reads_k0(sc):
        s.read(dst, addr, off)
    q0 = list(s.queue)
    body(s, sc, "steady", first=True)
    assert suffix(s.queue, q0)
    s.emit("s_cmp_eq_u32 %[iter], 0")
    s.emit("s_cbranch_scc1 L_w4_after_%=")
    s.emit("L_w4_loop_%=:")
    body(s, sc, "steady")
    assert suffix(s.queue, q0), "steady body must leave the LDS queue as it found it"
    s.emit("s_cbranch_scc1 L_w4_loop_%=")
    s.emit("L_w4_after_%=:")
    body(s, sc, "nodma")
    assert suffix(s.queue, q0)
    body(s, sc, "last")
    # every wave's LDS reads of this tile are retired (the last MFMAs consumed them): after
    # this barrier both buffers are free for the next tile's K-tiles 0 / 1
    s.emit("s_barrier")
    s.emit("s_cmp_eq_u32 %[has_next], 0")
    s.emit("s_cbranch_scc1 L_w4_end_%=")
    issue_two(s, "vn", sc)
    s.emit("L_w4_end_%=:")
    s.emit("s_nop 7")
    s.emit("s_nop 7")
    s.emit("s_nop 7")
    s.emit("s_mov_b32 m0, %[m0save]")
    return s.lines


def readout(i: int) -> list[str]:
    """v_accvgpr_read of accumulator row-block i (acc(i, 0..7), 32 AGPRs) into %0..%31."""
    return [f"v_accvgpr_read_b32 %{k}, a{32 * i + k}" for k in range(32)]


def render() -> str:
    out = ["// GENERATED by mlopamd/ops/gen_gemm_w4.py -- do not edit by hand.",
           "// The K-loop of gemm_w4_kernel (csrc/gemm_w4.hip): see the generator's docstring.",
           "#pragma once", ""]
    # one K-loop per count of VMEM ops issued after the prefetched K-tiles: plain and RoPE (32 x
    # 16-B stores per wave), SiLU-mul (16), and +2 for the row-scaled variants (W4_RS: two LDS-DMA
    # loads of the row sums of squares issued just before the K-loop)
    for si, sc in enumerate(SCHEDS):
        for ns in (32, 16, 34, 18):
            out.append(f"#define MLOP_W4_KLOOP_S{ns}_P{si}_ASM \\")
            for ln in kloop(ns, sc):
                out.append(f'  "{ln}\\n" \\')
            out.append('  ""')
            out.append("")
    # half-height tile: every epilogue issues half the stores (plain 16, SiLU-mul 8; +2 under W4_RS)
    for ns in (16, 8, 18, 10):
        out.append(f"#define MLOP_W4H_KLOOP_S{ns}_ASM \\")
        for ln in kloop(ns, SCHED_H):
            out.append(f'  "{ln}\\n" \\')
        out.append('  ""')
        out.append("")
    for i in range(8):
        out.append(f"#define MLOP_W4_READ{i}_ASM \\")
        for ln in readout(i):
            out.append(f'  "{ln}\\n" \\')
        out.append('  ""')
        out.append("")
    clob = ", ".join(f'"a{r}"' for r in range(256))
    out.append(f"#define MLOP_W4_AGPR_CLOBBERS {clob}")
    out.append("")
    return "\n".join(out)


def main():
    OUT.write_text(render())
    print(OUT)


if __name__ == "__main__":
    main()
