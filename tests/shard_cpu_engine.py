"""TEST INFRASTRUCTURE: a CPU stand-in for egraph.graph.Plan with the methods the partitioned
protocol (egraph/shard.py RankRun / run_partitioned) calls, built on the C oracle
(oracle/egraph_oracle.c: orc_hop_step, orc_topk).  It lets the N > 1 path -- partition, local
CSR, halo maps, all-gather exchange, top-k merge -- run under gloo on CPU; the HIP plan runs the
same protocol on the GPU (tests/test_shard_gpu.py).  Never imported by the package.
"""
from __future__ import annotations

import numpy as np
import torch

import oracle

NO_NODE = 0xFFFFFFFF


class CpuEngine:
    def __init__(self, lg, B: int, k: int):
        self.lg, self.B, self.k = lg, B, k
        self.V = len(lg.gid)
        self.padded_cols = B
        self.W = (B + 63) // 64
        self.owned = self.V
        self.x = None
        self.s0 = np.zeros((self.V, B), np.float32)
        self.hops_done = 0

    def set_owned(self, n):
        self.owned = n

    def set_seeds(self, lv, lc, ls):
        s0 = np.full((self.V, self.B), np.nan, np.float32)
        for v, c, s in zip(lv.tolist(), lc.tolist(), ls.tolist()):
            if v < self.V and c < self.B:
                cur = s0[v, c]
                s0[v, c] = s if np.isnan(cur) else np.fmax(cur, np.float32(s))
        self.s0 = np.nan_to_num(s0, nan=0.0).astype(np.float32)
        self.x = self.s0.copy()
        self.hops_done = 0

    def set_sources(self, src):
        self.R = np.zeros((self.V, self.B), bool)
        for b, v in enumerate(src.tolist()):
            if v < self.V:
                self.R[v, b] = True

    def hop(self):
        lg = self.lg
        self.x = oracle.hop_step(lg.row_ptr, lg.col, lg.val, self.x, self.s0)
        self.hops_done += 1

    def reach_hop(self):
        rp = self.lg.row_ptr.astype(np.int64)
        col = self.lg.col.astype(np.int64)
        new = self.R.copy()
        for v in range(self.V):
            if rp[v + 1] > rp[v]:
                new[v] |= self.R[col[rp[v]:rp[v + 1]]].any(axis=0)
        self.R = new

    # ---- exchange buffers (torch CPU tensors) ----
    def pack_scores(self, rows, out):
        r = rows.numpy().view(np.uint32)
        out[: len(r)] = torch.from_numpy(self.x[r])

    def unpack_scores(self, rows, src, inp):
        r, s = rows.numpy().view(np.uint32), src.numpy().view(np.uint32)
        self.x[r] = inp.numpy()[s]

    def _words(self, rows):
        bits = self.R[rows]
        pad = np.zeros((len(rows), self.W * 64), bool)
        pad[:, : self.B] = bits
        return np.packbits(pad.reshape(len(rows), self.W, 64)[:, :, ::-1], axis=2) \
            .view(">u8").reshape(len(rows), self.W).astype(np.uint64)

    def pack_reach(self, rows, out):
        r = rows.numpy().view(np.uint32)
        out[: len(r)] = torch.from_numpy(self._words(r).view(np.int64))

    def unpack_reach(self, rows, src, inp):
        r, s = rows.numpy().view(np.uint32), src.numpy().view(np.uint32)
        words = inp.numpy().view(np.uint64)[s]
        for j, v in enumerate(r.tolist()):
            for b in range(self.B):
                self.R[v, b] = bool((int(words[j, b // 64]) >> (b % 64)) & 1)

    def candidates(self, exclude_label):
        pass

    def topk(self, exclude_label):
        n = self.owned
        words = np.zeros((self.W, n), np.uint64)
        for b in range(self.B):
            words[b // 64] |= self.R[:n, b].astype(np.uint64) << np.uint64(b % 64)
        ids, sc = oracle.topk(np.ascontiguousarray(self.x[:n]), words, self.lg.vlabel[:n],
                              exclude_label, self.k)
        return torch.from_numpy(ids.view(np.int32)), torch.from_numpy(sc)

    def scores_owned(self):
        return self.x[: self.owned]

    # ---- the fixed-capacity sparse exchange (egr_plan_pack_sparse_cap / _unpack_sparse_cap) ----
    def _row_words(self, what, r):
        if what == "reach":
            return self._words(r).view(np.int64)                         # [n][W] words
        return self.x[r].view(np.int32).astype(np.int64) & 0xFFFFFFFF    # [n][B] value bits

    def pack_sparse_cap(self, what, rows, seg_dev, out, peer_cap, overflow, counts=None):
        r = rows.numpy().view(np.uint32)
        seg = seg_dev.numpy()
        vals = self._row_words(what, r)
        width = vals.shape[1] if vals.ndim == 2 else 0
        per = 2 if what == "reach" else 1
        stride = 1 + peer_cap * per               # header word (the entry count) + the entries
        o = out.numpy()
        for q in range(len(seg) - 1):
            ent = []
            for i in range(seg[q], seg[q + 1]):
                for b in np.flatnonzero(vals[i]).tolist():
                    ent.append(((i - seg[q]) * width + b, int(vals[i, b])))
            if len(ent) > peer_cap:
                overflow[0] = 1
            o[q * stride] = len(ent)              # entries, uncapped (the receiver clamps)
            if counts is not None:
                counts[q] = len(ent)
            ent = ent[:peer_cap]
            base = q * stride + 1
            for j, (idx, w) in enumerate(ent):
                if per == 2:
                    o[base + 2 * j], o[base + 2 * j + 1] = idx, w          # w: the signed word
                else:
                    o[base + j] = (idx << 32) | w

    def unpack_sparse_cap(self, what, recv_vertex, entries, peer_cap, rbase, overflow=None):
        rv = recv_vertex.numpy().view(np.uint32)
        e = entries.numpy()
        rb = rbase.numpy()
        per = 2 if what == "reach" else 1
        stride = 1 + peer_cap * per
        width = self.W if what == "reach" else self.padded_cols
        if what == "reach":
            self.R[rv] = False
        else:
            self.x[rv] = 0.0
        for s in range(len(rb)):
            n = int(e[s * stride])
            if n > peer_cap and overflow is not None:
                overflow[0] = 1
            for j in range(min(n, peer_cap)):
                if per == 2:
                    idx = int(e[s * stride + 1 + 2 * j])
                    w = int(e[s * stride + 2 + 2 * j]) & 0xFFFFFFFFFFFFFFFF
                else:
                    x = int(e[s * stride + 1 + j])
                    idx, w = x >> 32, x & 0xFFFFFFFF
                row = rv[rb[s] + idx // width]
                b = idx % width
                if what == "reach":
                    for t in range(64):
                        if b * 64 + t < self.B:
                            self.R[row, b * 64 + t] = bool((w >> t) & 1)
                else:
                    self.x[row, b] = np.array([w], np.uint32).view(np.float32)[0]
