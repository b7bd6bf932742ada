"""Step metadata for the ragged paged-attention kernel.

All int32 metadata of a step lives in ONE pinned host buffer with a fixed
layout and is shipped with ONE async H2D copy into ONE device buffer; the
kernel arguments are fixed views into it, so hipGraph-captured decode steps
see new values on every replay without re-capture.

Sequence-indexed arrays (q_start, q_len, ctx_len, block_tables) are indexed by
a stable *row* (the sequence's slot in [0, max_seqs)), so the host only
touches the rows that changed; tiles (16 MFMA q-rows = 16/G query tokens)
point at rows.  Rows with a prompt chunk of at least ``flash_min_q`` tokens
get flash-prefill tiles instead (128 q-rows = 128/G tokens each, ordered
longest-first over the whole step so the longest causal ranges start first).
"""
from __future__ import annotations

import os
from dataclasses import dataclass

import numpy as np
import torch

from .kv_cache import BLOCK_SIZE


@dataclass
class AttnMeta:
    positions: torch.Tensor   # int32 [T]
    slots: torch.Tensor       # int32 [T]
    block_tables: torch.Tensor  # int32 [max_seqs, max_blocks]
    tile_seq: torch.Tensor    # int32 [num_tiles]   decode-kernel tiles (16 q-rows)
    tile_q0: torch.Tensor     # int32 [num_tiles]
    ptile_seq: torch.Tensor   # int32 [num_ptiles]  flash-prefill tiles (128 q-rows)
    ptile_q0: torch.Tensor    # int32 [num_ptiles]
    q_start: torch.Tensor     # int32 [max_seqs]
    q_len: torch.Tensor       # int32 [max_seqs]
    ctx_len: torch.Tensor     # int32 [max_seqs]
    part_tokens: int
    nparts: int
    part_o: torch.Tensor
    part_ml: torch.Tensor
    logits_idx: torch.Tensor  # int64 [n_logits]
    num_tokens: int
    # int32 tickets (zero-initialised, re-armed by the kernel): the last partition of a
    # split-KV (tile, kv head) combines the slabs in the same launch; None -> reduce launch
    part_sem: torch.Tensor | None = None


# 128-token partitions: one 32-token page pair per wave at batch 1 (256: 312 tok/s, 128: 322,
# 64: 246 - the reduce pass and partial traffic grow faster than the parallelism; run38/39)
MIN_PART = 128
# workgroups a decode launch aims for before it splits contexts into partitions (2048 / 4096:
# batch 64 11,361 / 11,221 vs 11,643 tok/s at 1024, batch 16 flat: scripts/history/r4_twgs.sh);
# at most 2048, so tiles x kv heads x partitions stays within MetaBuffers.wp_capacity
TARGET_WGS = 1024


# flash-prefill tiles dispatched longest-first over the WHOLE step (LPT list scheduling), not
# sequence by sequence: a causal tile reads kv_end = ctx - q_len + q0 + 128/G keys, so with
# several prompts the per-sequence order put the last prompt's heaviest tiles behind most of
# the light ones and the launch ended on them (the tail of 4 x 2048 / 16 x 512,
# profiles/r06_flash_lpt.md).  The kv-head-fastest workgroup order inside a tile is unchanged.
# Only for steps with a prompt chunk of >= FLASH_LPT_MIN_Q tokens: measured on one box
# (scripts/bench_flash.py, ORDER=seq / lpt, interleaved) 4 x 2048 175 -> 166 us, 8 x 1024
# 110 -> 96 us, 1 x 8192 / 2 x 4096 unchanged, but 16 x 512 70 -> 74 us: short prompts lose more
# from the sequences' K / V pages interleaving in L2 than they gain in the tail.
# MLOP_FLASH_LPT=0: the per-sequence order (A/B switch).
FLASH_LPT = os.environ.get("MLOP_FLASH_LPT", "1") not in ("0", "false", "")
FLASH_LPT_MIN_Q = 1024


def order_flash_tiles(seq: np.ndarray, q0: np.ndarray, work: np.ndarray) -> None:
    """In place: (seq, q0) tile pairs sorted by descending ``work`` (keys read), ties in their
    given order (stable)."""
    o = np.argsort(-work, kind="stable")
    seq[:] = seq[o]
    q0[:] = q0[o]
    work[:] = work[o]


def plan_partitions(num_tiles: int, n_kv: int, max_ctx: int, min_part: int | None = None,
                    target_wgs: int | None = None) -> tuple[int, int]:
    """Split the KV range so a launch has >= ~target_wgs workgroups (256 CUs),
    partitions no shorter than ``min_part`` tokens; one partition when the batch
    already fills the chip (no reduce pass)."""
    min_part = MIN_PART if min_part is None else min_part
    target_wgs = TARGET_WGS if target_wgs is None else target_wgs
    max_ctx = max(32, max_ctx)
    base = max(1, num_tiles * n_kv)
    if base >= target_wgs // 2:
        return ((max_ctx + 31) // 32) * 32, 1
    nparts = max(1, min((max_ctx + min_part - 1) // min_part, (target_wgs + base - 1) // base))
    part = (max_ctx + nparts - 1) // nparts
    part = ((part + 31) // 32) * 32
    nparts = (max_ctx + part - 1) // part
    return part, nparts


class MetaBuffers:
    """Fixed-layout pinned host + device buffers for up to ``max_tokens`` tokens
    and ``max_seqs`` concurrent sequences."""

    def __init__(self, max_tokens: int, max_seqs: int, max_blocks_per_seq: int, group: int,
                 n_kv: int, max_model_len: int, device, flash_min_q: int = 17):
        self.device = torch.device(device)
        self.max_tokens, self.max_seqs, self.mb = max_tokens, max_seqs, max_blocks_per_seq
        self.G, self.n_kv, self.max_model_len = group, n_kv, max_model_len
        self.qt = 16 // group
        self.pqt = 128 // group if group <= 8 else 0  # flash tile tokens (0: no flash kernel for G > 8)
        self.flash_min_q = flash_min_q if self.pqt else 1 << 30
        self.max_tiles = max_tokens  # worst case: one tile per token
        self.npt = 0                 # flash tiles of the last fill
        self._pwork = np.zeros(self.max_tiles, dtype=np.int32)  # per flash tile: keys it reads
        sizes = [("positions", max_tokens), ("slots", max_tokens), ("tile_seq", self.max_tiles),
                 ("tile_q0", self.max_tiles), ("ptile_seq", self.max_tiles), ("ptile_q0", self.max_tiles),
                 ("q_start", max_seqs), ("q_len", max_seqs), ("ctx_len", max_seqs)]
        # ONE int32 buffer per side: [header | int32 metadata | ids (int64) | logits index (int64) |
        # block tables], every region 64-int aligned.  One H2D ships a step; a tensor-parallel
        # step is ONE broadcast of the device buffer (engine.StepSync: header + metadata + ids
        # together).  The block tables come last, so both move only the prefix up to the highest
        # row in use (extent()): [max_seqs, max_blocks] is most of the buffer at long contexts.
        self.HDR = 16
        self.off = {}
        o = self.HDR
        for name, n in sizes:
            self.off[name] = (o, n)
            o += (n + 63) // 64 * 64
        meta_hi = o
        ids_lo = o
        o += (2 * max_tokens + 63) // 64 * 64
        lidx_lo = o
        o += (2 * max_seqs + 63) // 64 * 64
        self.off["block_tables"] = (o, max_seqs * max_blocks_per_seq)
        o += (max_seqs * max_blocks_per_seq + 63) // 64 * 64
        self.total = o
        pin = self.device.type == "cuda"
        self.hbuf = torch.zeros(o, dtype=torch.int32, pin_memory=pin)
        self.dbuf = torch.zeros(o, dtype=torch.int32, device=self.device)
        self.hdr_h = self.hbuf[:self.HDR]
        self.hdr_hn = self.hdr_h.numpy()
        # metadata views keep their old names; offsets in self.off are into the whole buffer
        self.h, self.d = self.hbuf, self.dbuf
        self.hn = self.hbuf.numpy()
        self._meta_hi = meta_hi
        self.ids_h = self.hbuf[ids_lo:ids_lo + 2 * max_tokens].view(torch.int64)
        self.ids_hn = self.ids_h.numpy()
        self.ids_d = self.dbuf[ids_lo:ids_lo + 2 * max_tokens].view(torch.int64)
        self.lidx_h = self.hbuf[lidx_lo:lidx_lo + 2 * max_seqs].view(torch.int64)
        self.lidx_hn = self.lidx_h.numpy()
        self.lidx_d = self.dbuf[lidx_lo:lidx_lo + 2 * max_seqs].view(torch.int64)
        # partial-softmax workspace for the split-KV path (sized for the worst launch)
        # plan_partitions only splits launches with < target/2 base workgroups, so
        # tiles * n_kv * nparts stays <= ~2 * target: size for 4096 partial tiles
        self.wp_capacity = 4096
        self.part_o = torch.empty(self.wp_capacity * 16 * 128, dtype=torch.float32, device=self.device)
        self.part_ml = torch.empty(self.wp_capacity * 16 * 2, dtype=torch.float32, device=self.device)
        self.part_sem = torch.zeros(self.wp_capacity, dtype=torch.int32, device=self.device)
        bt = self.view_h("block_tables").reshape(max_seqs, max_blocks_per_seq)
        self.bt_h = bt  # numpy view [max_seqs, mb]

    def view_h(self, name):
        o, n = self.off[name]
        return self.hn[o:o + n]

    def view_d(self, name, n=None):
        o, cap = self.off[name]
        return self.d[o:o + (cap if n is None else n)]

    def extent(self, rows_hi: int | None = None) -> int:
        """int32 words of the buffer a step needs: everything up to block-table row ``rows_hi``
        (the engine's high-water row: graph-padding rows attend to nothing and read no block
        table), a multiple of 64 words; None = the whole buffer."""
        if rows_hi is None:
            return self.total
        o, _ = self.off["block_tables"]
        return min(self.total, o + (max(0, rows_hi) * self.mb + 63) // 64 * 64)

    def upload(self, n_ids: int = 0, n_logits: int = 0, rows_hi: int | None = None):
        """ONE async H2D of header + metadata + ids + logits index (+ the block-table rows in
        use) on the current stream."""
        n = self.extent(rows_hi)
        self.dbuf[:n].copy_(self.hbuf[:n], non_blocking=True)

    def set_header(self, vals) -> None:
        self.hdr_hn[:len(vals)] = vals

    def meta(self, num_tokens: int, num_tiles: int, n_logits: int, part_tokens: int, nparts: int,
             num_ptiles: int = 0) -> AttnMeta:
        if nparts > 1:
            assert num_tiles * self.n_kv * nparts <= self.wp_capacity, "partial workspace too small"
        return AttnMeta(
            positions=self.view_d("positions", num_tokens), slots=self.view_d("slots", num_tokens),
            block_tables=self.view_d("block_tables").view(self.max_seqs, self.mb),
            tile_seq=self.view_d("tile_seq", num_tiles), tile_q0=self.view_d("tile_q0", num_tiles),
            ptile_seq=self.view_d("ptile_seq", num_ptiles), ptile_q0=self.view_d("ptile_q0", num_ptiles),
            q_start=self.view_d("q_start"), q_len=self.view_d("q_len"), ctx_len=self.view_d("ctx_len"),
            part_tokens=part_tokens, nparts=nparts, part_o=self.part_o, part_ml=self.part_ml,
            logits_idx=self.lidx_d[:n_logits], num_tokens=num_tokens, part_sem=self.part_sem)

    def fill(self, rows, q_lens, ctx_lens, token_ids_per_seq, want_logits=None):
        """Fill host arrays for a ragged batch.

        rows[i]: the row slot of batch sequence i; q_lens[i] new tokens whose
        KV is written this step; ctx_lens[i] context length AFTER this step;
        token_ids_per_seq[i]: the q_len input ids. Block tables must already
        hold the pages covering ctx_lens.  want_logits[i] (default all): emit a
        logits row for sequence i's last token.  Returns (T, num_tiles, n_logits);
        the flash-tile count is left in ``self.npt``."""
        return self._fill_ragged(0, 0, 0, rows, q_lens, ctx_lens, token_ids_per_seq, want_logits)

    def fill_mixed(self, d_rows: np.ndarray, d_ctx: np.ndarray, d_last: np.ndarray,
                   rows, q_lens, ctx_lens, token_ids_per_seq, want_logits=None):
        """One step that decodes ``d_rows`` (one token each, vectorised, first B
        tokens / tiles / logits) and prefills chunks of other sequences after
        them (Sarathi-style mixed batch: the decode rows ride in the prefill's
        GEMMs).  Returns (T, num_tiles, n_logits)."""
        B = len(d_rows)
        self.fill_decode(d_rows, d_ctx, d_last, pad_to=B)
        return self._fill_ragged(B, B, B, rows, q_lens, ctx_lens, token_ids_per_seq, want_logits)

    def _fill_ragged(self, t, nt, nl, rows, q_lens, ctx_lens, token_ids_per_seq, want_logits):
        pos_h, slot_h = self.view_h("positions"), self.view_h("slots")
        ts_h, tq_h = self.view_h("tile_seq"), self.view_h("tile_q0")
        pts_h, ptq_h = self.view_h("ptile_seq"), self.view_h("ptile_q0")
        npt, pqt = 0, self.pqt
        max_flash_q = 0
        qs_h, ql_h, cl_h = self.view_h("q_start"), self.view_h("q_len"), self.view_h("ctx_len")
        qt = self.qt
        for i, row in enumerate(rows):
            ql, cl = int(q_lens[i]), int(ctx_lens[i])
            qs_h[row], ql_h[row], cl_h[row] = t, ql, cl
            p = np.arange(cl - ql, cl, dtype=np.int32)
            pos_h[t:t + ql] = p
            slot_h[t:t + ql] = self.bt_h[row, p // BLOCK_SIZE] * BLOCK_SIZE + p % BLOCK_SIZE
            self.ids_hn[t:t + ql] = token_ids_per_seq[i]
            if ql >= self.flash_min_q:
                n = (ql + pqt - 1) // pqt
                pts_h[npt:npt + n] = row
                ptq_h[npt:npt + n] = np.arange(n - 1, -1, -1, dtype=np.int32) * pqt  # latest first
                self._pwork[npt:npt + n] = (cl - ql + pqt) + ptq_h[npt:npt + n]  # keys each tile reads
                max_flash_q = max(max_flash_q, ql)
                npt += n
            else:
                ntile = (ql + qt - 1) // qt
                ts_h[nt:nt + ntile] = row
                tq_h[nt:nt + ntile] = np.arange(ntile, dtype=np.int32) * qt
                nt += ntile
            t += ql
            if want_logits is None or want_logits[i]:
                self.lidx_hn[nl] = t - 1
                nl += 1
        if npt > 1 and FLASH_LPT and max_flash_q >= FLASH_LPT_MIN_Q:
            order_flash_tiles(pts_h[:npt], ptq_h[:npt], self._pwork[:npt])
        self.npt = npt
        return t, nt, nl

    def fill_decode(self, rows: np.ndarray, ctx_lens: np.ndarray, last_tokens: np.ndarray, pad_to: int):
        """Vectorised decode fill: one query token per sequence, padded to the
        graph bucket ``pad_to`` with rows that attend to nothing."""
        B = len(rows)
        self.npt = 0
        pos_h, slot_h = self.view_h("positions"), self.view_h("slots")
        ts_h, tq_h = self.view_h("tile_seq"), self.view_h("tile_q0")
        qs_h, ql_h, cl_h = self.view_h("q_start"), self.view_h("q_len"), self.view_h("ctx_len")
        p = (ctx_lens - 1).astype(np.int32)
        pos_h[:B] = p
        slot_h[:B] = self.bt_h[rows, p // BLOCK_SIZE] * BLOCK_SIZE + p % BLOCK_SIZE
        ts_h[:B] = rows
        tq_h[:B] = 0
        qs_h[rows] = np.arange(B, dtype=np.int32)
        ql_h[rows] = 1
        cl_h[rows] = ctx_lens
        self.ids_hn[:B] = last_tokens
        self.lidx_hn[:B] = np.arange(B)  # the identity: decode graphs skip the gather (Engine.capture_graphs)
        if pad_to > B:
            pad_rows = self.pad_rows(pad_to - B)
            pos_h[B:pad_to] = 0
            slot_h[B:pad_to] = -1
            ts_h[B:pad_to] = pad_rows
            tq_h[B:pad_to] = 0
            qs_h[pad_rows] = np.arange(B, pad_to, dtype=np.int32)
            ql_h[pad_rows] = 1
            cl_h[pad_rows] = 0
            self.ids_hn[B:pad_to] = 0
            self.lidx_hn[B:pad_to] = np.arange(B, pad_to)

    def pad_rows(self, n: int) -> np.ndarray:
        """Rows reserved for graph padding: the top of the row space (never handed to sequences)."""
        return np.arange(self.max_seqs - n, self.max_seqs, dtype=np.int32)
