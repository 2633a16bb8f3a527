"""Edge-cut partitioned evidence graphs with a per-hop halo exchange (BASELINE
config C4: graphs too large for one GPU).

Partition.  Workload vertices (Pod / Deployment / Service / Event / LogPattern / MetricAnomaly /
ChangeEvent / Incident) are cut into contiguous ranges of vertex ids balanced by CSR entries;
the generator and the collectors lay vertices out namespace by namespace, so a range is a run of
whole namespaces and only the cross-namespace edges (CALLS, SCHEDULED_ON) are cut.  Kubernetes
`Node` vertices, whose pods come from every namespace, are spread by a hash of their id.

Local graph of rank r.  Owned vertices first, in global order, with their FULL rows (entries
remapped to local ids, CSR order kept, so every row's fmaf chain is exactly the unpartitioned
one); then the halo (non-owned neighbours of owned vertices), in global order, with empty rows.
Rank r sends q the r-owned rows that q's rows read.

Per hop (run_partitioned): the engine computes its rows; the fresh rows other ranks read are
packed (one contiguous segment per reader) and exchanged point-to-point (RCCL over xGMI:
torch.distributed all_to_all_single with per-peer counts), then unpacked into the halo rows.
The default exchange is SPARSE: only the non-zero entries of the packed rows cross the link
(a boundary row is non-zero only in the columns whose 3-hop frontier reached it), as
(index, value) int64 words after a per-peer count exchange; the dense exchange ([rows][Bpad]
fp32 for scores, [rows][ceil(B/64)] u64 for reach) remains as run_partitioned(sparse=False).  After the last hop each rank ranks its owned candidates; the (score, global id)
lists are all-gathered and merged (score desc, global id asc) -- the unpartitioned top-k.
Scores, reach sets and top-k are bit-identical to the single-GPU plan (tests/test_shard*.py).
"""
from __future__ import annotations

import contextlib

from dataclasses import dataclass

import numpy as np
import torch

NO_NODE = 0xFFFFFFFF


def partition_vertices(row_ptr: np.ndarray, vlabel: np.ndarray, label_names: list[str], P: int,
                       hash_labels: tuple[str, ...] = ("Node",)) -> np.ndarray:
    """owner[v] in [0, P): hashed for `hash_labels`, contiguous ranges otherwise, balanced so
    that every rank's total row weight (degree + 1: a dense hop writes a row and gathers its
    entries) -- its hashed vertices' included -- is as equal as the ranges allow."""
    V = len(row_ptr) - 1
    if P < 1:
        raise ValueError("P must be >= 1")
    owner = np.zeros(V, np.int32)
    if P == 1:
        return owner
    hashed = np.isin(vlabel, [label_names.index(n) for n in hash_labels if n in label_names])
    deg = np.diff(row_ptr.astype(np.int64))
    ids = np.flatnonzero(hashed).astype(np.uint64)
    hown = (((ids * np.uint64(0x9E3779B1)) >> np.uint64(7)) % np.uint64(P)).astype(np.int64)
    # the hashed vertices' weight per rank, then each rank's share of the contiguous weight:
    # what brings it to the common target (never negative)
    hw = np.bincount(hown, weights=deg[hashed] + 1, minlength=P) if len(ids) else np.zeros(P)
    w = np.where(hashed, 0, deg + 1)            # +1: isolated vertices still weigh something
    cum = np.cumsum(w)
    total = float(cum[-1]) if V else 0.0
    target = (total + hw.sum()) / P
    cap = np.maximum(target - hw, 0.0)
    cap *= total / max(cap.sum(), 1e-9)         # (the contiguous weight, all of it, is assigned)
    bounds = np.cumsum(cap)[:-1]
    owner[:] = np.minimum(np.searchsorted(bounds, cum - 0.5, side="right"), P - 1).astype(np.int32)
    owner[hashed] = hown.astype(np.int32)
    return owner


@dataclass
class LocalGraph:
    rank: int
    P: int
    gid: np.ndarray          # local -> global vertex id (owned, then halo)
    n_owned: int
    row_ptr: np.ndarray      # local CSR, u32
    col: np.ndarray
    meta: np.ndarray
    val: np.ndarray
    vlabel: np.ndarray
    send_rows: np.ndarray    # local ids (owned) sent each hop, grouped by destination rank
    send_counts: list        # rows sent to rank q (send_rows[sum(send_counts[:q]):...])
    recv_counts: list        # rows received from rank q
    halo_rows: np.ndarray    # local ids of the halo rows
    halo_src: np.ndarray     # per halo row: its row in the received buffer


def build_local(csr: dict, vlabel: np.ndarray, owner: np.ndarray, rank: int, P: int) -> LocalGraph:
    """Rank `rank`'s local CSR and exchange maps from the global host CSR (graph.csr()).

    The halo exchange is point-to-point (all-to-all): rank r sends rank q exactly the rows of
    r-owned vertices that q's rows read, in global id order, and q receives them grouped by
    sender -- so each boundary row crosses xGMI once per reader instead of once per rank."""
    rp = csr["row_ptr"].astype(np.int64)
    col = csr["col"].astype(np.int64)
    V = len(rp) - 1
    deg = np.diff(rp)
    src_of = np.repeat(np.arange(V, dtype=np.int64), deg)
    cross = owner[src_of] != owner[col]         # entry (v -> u) across ranks: u is in v's halo
    # (reader rank, vertex) pairs, unique, sorted by reader then vertex id
    pairs = np.unique(owner[src_of[cross]].astype(np.int64) * V + col[cross])
    reader, vert = pairs // V, pairs % V
    owned = np.flatnonzero(owner == rank)
    halo = vert[reader == rank]                 # sorted by global id
    gid = np.concatenate([owned, halo]).astype(np.int64)
    g2l = np.full(V, -1, np.int64)
    g2l[gid] = np.arange(len(gid))
    # owned rows in global order keep their full rows (CSR order preserved)
    starts, ends = rp[owned], rp[owned + 1]
    n_ent = ends - starts
    l_rp = np.zeros(len(gid) + 1, np.int64)
    l_rp[1:len(owned) + 1] = np.cumsum(n_ent)
    l_rp[len(owned) + 1:] = l_rp[len(owned)]
    take = np.concatenate([np.arange(s, e) for s, e in zip(starts, ends)]) if len(owned) else \
        np.zeros(0, np.int64)
    # sends: pairs whose vertex this rank owns, grouped by reader (already sorted that way)
    mine = owner[vert] == rank
    send_v = vert[mine]
    send_counts = np.bincount(reader[mine], minlength=P).astype(np.int64).tolist()
    # receives: the halo grouped by owner, vertex order within a group
    h_owner = owner[halo].astype(np.int64)
    recv_order = np.lexsort((halo, h_owner))
    recv_counts = np.bincount(h_owner, minlength=P).astype(np.int64).tolist()
    halo_src = np.empty(len(halo), np.int64)
    halo_src[recv_order] = np.arange(len(halo))
    return LocalGraph(
        rank=rank, P=P, gid=gid, n_owned=len(owned),
        row_ptr=l_rp.astype(np.uint32), col=g2l[col[take]].astype(np.uint32),
        meta=csr["meta"][take].astype(np.uint8), val=csr["val"][take].astype(np.float32),
        vlabel=vlabel[gid].astype(np.uint8),
        send_rows=g2l[send_v].astype(np.uint32), send_counts=send_counts, recv_counts=recv_counts,
        halo_rows=np.arange(len(owned), len(gid), dtype=np.uint32),
        halo_src=halo_src.astype(np.uint32))


def local_seeds(lg: LocalGraph, V: int, sv: np.ndarray, sc: np.ndarray, ss: np.ndarray):
    """The seed triples of owned and halo vertices, in local ids (halo seeds are read by owned
    rows in the first hop)."""
    g2l = np.full(V, -1, np.int64)
    g2l[lg.gid] = np.arange(len(lg.gid))
    lv = g2l[sv.astype(np.int64)] if len(sv) else np.zeros(0, np.int64)
    keep = lv >= 0
    return lv[keep].astype(np.uint32), sc[keep].astype(np.uint32), ss[keep].astype(np.float32)


def local_sources(lg: LocalGraph, V: int, src: np.ndarray) -> np.ndarray:
    g2l = np.full(V + 1, -1, np.int64)
    g2l[lg.gid] = np.arange(len(lg.gid))
    s = src.astype(np.int64)
    s = np.where((s >= 0) & (s < V), s, V)
    out = g2l[s]
    return np.where(out >= 0, out, NO_NODE).astype(np.uint32)


class TorchComm:
    """Collectives across the process group.  RCCL on device buffers is the production path (one
    process per GPU): all_to_all_single with per-peer row counts for the halo, all_gather for the
    candidate lists.  Under gloo (CPU tests, or several processes sharing one GPU, which RCCL
    refuses) the buffers are staged through host memory."""

    def __init__(self, group=None):
        import torch.distributed as dist
        self.dist = dist
        self.group = group
        self.P = dist.get_world_size(group)
        self.gloo = dist.get_backend(group) == "gloo"
        self.calls = 0          # collectives issued (each all_to_all_v is two: counts, then data)

    def all_gather(self, send: list[torch.Tensor]) -> list[torch.Tensor]:
        (x,) = send
        x = x.contiguous()
        self.calls += 1
        if self.gloo:
            h = x.cpu()
            parts = [torch.empty_like(h) for _ in range(self.P)]
            self.dist.all_gather(parts, h, group=self.group)
            return [torch.cat(parts).to(x.device)]
        out = torch.empty((self.P * x.shape[0],) + tuple(x.shape[1:]), dtype=x.dtype, device=x.device)
        self.dist.all_gather_into_tensor(out, x, group=self.group)
        return [out]

    def all_to_all(self, items: list) -> None:
        """items = [(send, send_counts, recv, recv_counts)] for this process's one rank; rows
        send[off_q : off_q + send_counts[q]] go to rank q, recv is filled grouped by sender."""
        ((send, sc, recv, rc),) = items
        self.calls += 1
        if self.gloo:
            hs, hr = send.cpu(), torch.empty(recv.shape, dtype=recv.dtype)
            self.dist.all_to_all_single(hr, hs, output_split_sizes=rc, input_split_sizes=sc,
                                        group=self.group)
            recv.copy_(hr)
            return
        self.dist.all_to_all_single(recv, send, output_split_sizes=rc, input_split_sizes=sc,
                                    group=self.group)

    def all_to_all_v(self, items: list) -> list:
        """items = [(send 1-D int64, send_counts)] for this process's one rank -> [recv, with
        the per-sender counts]: sizes are exchanged first (one int64 per peer), then the data."""
        ((send, sc),) = items
        dev = send.device
        self.calls += 2
        cnt = torch.tensor(sc, dtype=torch.int64)
        rcnt = torch.empty(self.P, dtype=torch.int64)
        if self.gloo:
            self.dist.all_to_all_single(rcnt, cnt, group=self.group)
        else:
            rc_d = torch.empty(self.P, dtype=torch.int64, device=dev)
            self.dist.all_to_all_single(rc_d, cnt.to(dev), group=self.group)
            rcnt = rc_d.cpu()
        rc = rcnt.tolist()
        recv = torch.empty(sum(rc), dtype=send.dtype, device=dev)
        if self.gloo:
            hr = torch.empty(sum(rc), dtype=send.dtype)
            self.dist.all_to_all_single(hr, send.cpu(), output_split_sizes=rc, input_split_sizes=sc,
                                        group=self.group)
            recv.copy_(hr)
        else:
            self.dist.all_to_all_single(recv, send, output_split_sizes=rc, input_split_sizes=sc,
                                        group=self.group)
        return [(recv, rc)]


    def all_to_all_fixed(self, items: list) -> None:
        """items = [(send, recv)]: equal splits -- block q of send (numel / P) goes to rank q and
        block r of recv comes from rank r.  No split sizes, so nothing is read on the host."""
        ((send, recv),) = items
        self.calls += 1
        if self.gloo:
            hr = torch.empty(recv.shape, dtype=recv.dtype)
            self.dist.all_to_all_single(hr, send.cpu(), group=self.group)
            recv.copy_(hr)
            return
        self.dist.all_to_all_single(recv, send, group=self.group)

    def any_flag(self, flags: list) -> bool:
        """True if any rank's flag tensor (device int32 [1]) is non-zero (one all-reduce and one
        host read per call)."""
        (f,) = flags
        self.calls += 1
        t = f.to(torch.int64).clone() if not self.gloo else f.to(torch.int64).cpu()
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX, group=self.group)
        return bool(t.item())


class LocalComm:
    """All ranks in one process (tests, and a multi-partition single-GPU run): gathers are
    concatenations, the all-to-all copies each sender's segment into its reader's buffer.
    `calls` counts the collectives the P ranks would issue (one per call, as TorchComm)."""

    def __init__(self):
        self.calls = 0

    def all_gather(self, send: list[torch.Tensor]) -> list[torch.Tensor]:
        self.calls += 1
        cat = torch.cat([s.to(send[0].device) for s in send])
        return [cat.to(s.device) for s in send]

    def all_to_all(self, items: list) -> None:
        self.calls += 1
        P = len(items)
        s_off = [np.concatenate([[0], np.cumsum(sc)]) for _, sc, _, _ in items]
        r_off = [np.concatenate([[0], np.cumsum(rc)]) for _, _, _, rc in items]
        for q in range(P):                       # reader
            for r in range(P):                   # sender
                n = items[r][1][q]
                assert n == items[q][3][r]
                if n:
                    items[q][2][r_off[q][r]: r_off[q][r] + n] = \
                        items[r][0][s_off[r][q]: s_off[r][q] + n].to(items[q][2].device)


    def all_to_all_fixed(self, items: list) -> None:
        self.calls += 1
        P = len(items)
        for q in range(P):                       # reader
            recv = items[q][1]
            bq = recv.numel() // P
            for r in range(P):                   # sender
                send = items[r][0]
                bs = send.numel() // P
                assert bs == bq
                recv[r * bq:(r + 1) * bq] = send[q * bs:(q + 1) * bs].to(recv.device)

    def any_flag(self, flags: list) -> bool:
        self.calls += 1
        return any(bool(f.item()) for f in flags)

    def all_to_all_v(self, items: list) -> list:
        self.calls += 2
        P = len(items)
        s_off = [np.concatenate([[0], np.cumsum(sc)]) for _, sc in items]
        out = []
        for q in range(P):
            parts = [items[r][0][s_off[r][q]: s_off[r][q] + items[r][1][q]].to(items[q][0].device)
                     for r in range(P)]
            out.append((torch.cat(parts), [items[r][1][q] for r in range(P)]))
        return out


class RankRun:
    """One rank's part of a partitioned pass.  `engine` is the HIP Plan of the local snapshot
    (egraph.graph.Plan); any object with the same methods works (the CPU tests use the oracle)."""

    def __init__(self, lg: LocalGraph, engine, device):
        self.lg, self.eng, self.dev = lg, engine, device
        self.send = torch.from_numpy(lg.send_rows.view(np.int32)).to(device)
        self.halo = torch.from_numpy(lg.halo_rows.view(np.int32)).to(device)
        self.src = torch.from_numpy(lg.halo_src.view(np.int32)).to(device)
        self.gid = torch.from_numpy(lg.gid).to(device)
        B = engine.B
        self.Bpad = engine.padded_cols
        self.W = (B + 63) // 64
        ns, nr = len(lg.send_rows), len(lg.halo_rows)
        self._dense = None         # dense exchange buffers, allocated on first use
        self.sent_bytes = 0        # bytes this rank put on the wire (every exchange so far)
        # per exchange, the largest transfer to ONE peer (xGMI is point to point: the peers'
        # transfers run on separate links at once, so this is what an exchange waits for)
        self.link_bytes = 0
        self.exchanges = 0
        # sparse exchange: the local vertex of each received row (rows grouped by sender) and
        # each sender's first received row
        rv = np.zeros(nr, np.uint32)
        rv[lg.halo_src.astype(np.int64)] = lg.halo_rows
        self.recv_vertex = torch.from_numpy(rv.view(np.int32)).to(device)
        self.recv_base = torch.from_numpy(_seg_starts(lg.recv_counts)[:-1]).to(device)
        self.send_seg = _seg_starts(lg.send_counts)
        self._sx = {}              # sparse send buffers (int64 words), grown on demand
        # fixed-capacity exchange (run_partitioned(fixed=True)): entries per peer slot per kind,
        # sized from a calibrating pass over the host-count path; slot buffers; overflow flag
        self.seg_dev = torch.from_numpy(self.send_seg).to(device)
        self.cap: dict = {}
        self.max_seen: dict = {}
        self._fx: dict = {}
        self.overflow = torch.zeros(1, dtype=torch.int32, device=device)
        self.overflows = 0         # passes that overflowed a slot (and were re-run)
        engine.set_owned(lg.n_owned)

    def _dense_bufs(self):
        if self._dense is None:
            ns, nr, dev = len(self.lg.send_rows), len(self.lg.halo_rows), self.send.device
            self._dense = (torch.zeros((ns, self.Bpad), dtype=torch.float32, device=dev),
                           torch.zeros((nr, self.Bpad), dtype=torch.float32, device=dev),
                           torch.zeros((ns, self.W), dtype=torch.int64, device=dev),
                           torch.zeros((nr, self.W), dtype=torch.int64, device=dev))
        return self._dense

    send_s = property(lambda self: self._dense_bufs()[0])   # [rows][Bpad] fp32 scores
    recv_s = property(lambda self: self._dense_bufs()[1])
    send_r = property(lambda self: self._dense_bufs()[2])   # [rows][W] reach words
    recv_r = property(lambda self: self._dense_bufs()[3])

    @property
    def halo_bytes_per_hop(self) -> int:
        """Bytes this rank sends per hop with the dense exchange (scores + reach words)."""
        return len(self.lg.send_rows) * (self.Bpad * 4 + self.W * 8)




def _max_peer(r: "RankRun", per_peer: list) -> int:
    """The largest of the bytes a rank sends to each OTHER rank in one exchange."""
    return max((b for q, b in enumerate(per_peer) if q != r.lg.rank), default=0)


def _seg_starts(counts) -> np.ndarray:
    return np.concatenate([[0], np.cumsum(counts)]).astype(np.int64)


class HaloOverflow(RuntimeError):
    """A fixed-capacity halo exchange had more non-zero entries for a peer than its slot holds:
    the pass's results are incomplete and it must be run again (the slots have been grown)."""


def _slot_words(what: str, cap: int) -> int:
    """One peer slot of the fixed-capacity exchange: a header word (the sender's entry count
    for that peer), then cap entries of one (scores) or two (reach) int64 words."""
    return 1 + cap * (2 if what == "reach" else 1)


def _fixed_bufs(r: "RankRun", what: str):
    P = r.lg.P
    cap = r.cap[what]
    b = r._fx.get(what)
    if b is None or b[0] != cap:
        dev = r.send.device
        n = P * _slot_words(what, cap)
        b = r._fx[what] = (cap,
                           torch.empty(n, dtype=torch.int64, device=dev),     # send slots
                           torch.empty(n, dtype=torch.int64, device=dev))     # recv slots
    return b


def _exchange_fixed(runs: list[RankRun], comm, what: str) -> None:
    """The sparse halo exchange with fixed-capacity peer slots: device pack (each slot headed by
    its entry count; overflow stays on the device), ONE equal-split all-to-all of the slots,
    device unpack (a header past the capacity sets the receiver's overflow flag too) -- no host
    synchronisation per exchange (egr_plan_pack_sparse_cap)."""
    items = []
    for r in runs:
        cap, sbuf, rbuf = _fixed_bufs(r, what)
        r.eng.pack_sparse_cap(what, r.send, r.seg_dev, sbuf, cap, r.overflow)
        r.sent_bytes += 8 * len(r.lg.send_counts) * _slot_words(what, cap)
        r.link_bytes += 8 * _slot_words(what, cap) if r.lg.P > 1 else 0
        r.exchanges += 1
        items.append((sbuf, rbuf))
    comm.all_to_all_fixed(items)
    for r in runs:
        cap, _, rbuf = _fixed_bufs(r, what)
        r.eng.unpack_sparse_cap(what, r.recv_vertex, rbuf, cap, r.recv_base, r.overflow)


def _exchange_sparse(runs: list[RankRun], comm, what: str) -> None:
    """The halo exchange with only the NON-ZERO entries on the wire (module doc).  Engines
    with native sparse packing (the HIP plan: egr_plan_pack_sparse / unpack_sparse) pack and
    scatter on the device; other engines (the CPU test engine) go through _exchange_sparse_py,
    the same entries built with tensor ops."""
    if not all(hasattr(r.eng, "pack_sparse") for r in runs):
        return _exchange_sparse_py(runs, comm, what)
    items = []
    for r in runs:
        ns = len(r.lg.send_rows)
        width = r.W if what == "reach" else r.Bpad
        per = 2 if what == "reach" else 1
        buf = r._sx.get(what)
        cap = ns * width * per
        if buf is None or buf.numel() < max(cap, 1):
            buf = r._sx[what] = torch.empty(max(cap, 1), dtype=torch.int64, device=r.send.device)
        counts = r.eng.pack_sparse(what, r.send, r.send_seg, buf)
        r.max_seen[what] = max(r.max_seen.get(what, 0), max(counts, default=0))
        n_words = [per * c for c in counts]
        r.sent_bytes += 8 * sum(n_words) + 8 * len(counts)
        r.link_bytes += _max_peer(r, [8 * w + 8 for w in n_words])
        r.exchanges += 1
        items.append((buf[: sum(n_words)], n_words))
    out = comm.all_to_all_v(items)
    for r, (recv, rc) in zip(runs, out):
        per = 2 if what == "reach" else 1
        eseg = torch.from_numpy(_seg_starts([c // per for c in rc])).to(recv.device)
        r.eng.unpack_sparse(what, r.recv_vertex, recv, eseg, r.recv_base)


def _exchange_sparse_py(runs: list[RankRun], comm, what: str) -> None:
    """The halo exchange with only the NON-ZERO entries on the wire: a boundary row's scores
    are non-zero only in the columns whose frontier reached it, and its reach words only where
    a column reached it.  Each rank packs its send rows (device-local), keeps the non-zero
    (row-in-segment, column) entries as one int64 each -- index << 32 | value bits (scores) or
    index + word (reach, two int64) -- exchanges the per-peer counts, then the entries, and
    scatters them into its zeroed halo rows.  Bit-identical to the dense exchange."""
    items, meta = [], []
    for r in runs:
        if what == "scores":
            r.eng.pack_scores(r.send, r.send_s)
            buf, width = r.send_s, r.Bpad
        else:
            r.eng.pack_reach(r.send, r.send_r)
            buf, width = r.send_r, r.W
        flat = buf.view(-1)
        nz = torch.nonzero(flat, as_tuple=True)[0]               # row-major: grouped by peer
        row = nz // width
        seg = _seg_starts(r.lg.send_counts)
        seg_t = torch.from_numpy(seg).to(nz.device)
        peer = torch.searchsorted(seg_t[1:], row, right=True)
        local = (row - seg_t[peer]) * width + (nz % width)       # index inside the peer's segment
        counts = torch.bincount(peer, minlength=len(r.lg.send_counts)).cpu().tolist()
        r.max_seen[what] = max(r.max_seen.get(what, 0), max(counts, default=0))   # (slot calibration)
        if what == "scores":
            if int(np.diff(seg).max(initial=0)) * width >= 1 << 32:
                raise ValueError("sparse score exchange: a peer segment's (row, column) index "
                                 "exceeds 2^32 (rows x columns); use the dense halo")
            vbits = flat[nz].view(torch.int32).to(torch.int64) & 0xFFFFFFFF
            payload = (local << 32) | vbits
            n_per = [c for c in counts]
        else:
            payload = torch.stack([local, flat[nz]], dim=1).reshape(-1)
            n_per = [2 * c for c in counts]
        r.sent_bytes += int(payload.numel()) * 8 + 8 * len(counts)
        r.link_bytes += _max_peer(r, [8 * w + 8 for w in n_per])
        r.exchanges += 1
        items.append((payload.contiguous(), n_per))
        meta.append(width)
    out = comm.all_to_all_v(items)
    for r, (recv, rc), width in zip(runs, out, meta):
        dst = r.recv_s if what == "scores" else r.recv_r
        dst.zero_()
        roff = _seg_starts(r.lg.recv_counts)
        base = torch.from_numpy(np.repeat(roff[:-1] * width,
                                          [c // (1 if what == "scores" else 2) for c in rc])).to(dst.device)
        if what == "scores":
            idx = (recv >> 32) + base
            dst.view(-1)[idx] = (recv & 0xFFFFFFFF).to(torch.int32).view(torch.float32)
        else:
            pairs = recv.view(-1, 2)
            dst.view(-1)[pairs[:, 0] + base] = pairs[:, 1]
        if what == "scores":
            r.eng.unpack_scores(r.halo, r.src, r.recv_s)
        else:
            r.eng.unpack_reach(r.halo, r.src, r.recv_r)


def _exchange(runs: list[RankRun], comm, what: str) -> None:
    items = []
    for r in runs:
        if what == "scores":
            r.eng.pack_scores(r.send, r.send_s)
            items.append((r.send_s, r.lg.send_counts, r.recv_s, r.lg.recv_counts))
        else:
            r.eng.pack_reach(r.send, r.send_r)
            items.append((r.send_r, r.lg.send_counts, r.recv_r, r.lg.recv_counts))
    comm.all_to_all(items)
    for r in runs:
        row_b = r.Bpad * 4 if what == "scores" else r.W * 8
        r.sent_bytes += len(r.lg.send_rows) * row_b
        r.link_bytes += _max_peer(r, [int(c) * row_b for c in r.lg.send_counts])
        r.exchanges += 1
        if what == "scores":
            r.eng.unpack_scores(r.halo, r.src, r.recv_s)
        else:
            r.eng.unpack_reach(r.halo, r.src, r.recv_r)


_SIDE: dict = {}


def _side_stream(dev: torch.device):
    """The second stream the reach chain runs on (one per device, created once)."""
    st = _SIDE.get(dev.index)
    if st is None:
        st = _SIDE[dev.index] = torch.cuda.Stream(dev)
    return st


def run_partitioned(runs: list[RankRun], comm, hops: int, exclude_label: int, k: int,
                    sparse: bool = True, fixed: bool = False, overlap: bool | None = None):
    """`hops` hops of propagation and reach on every local rank in `runs` (seeds and sources
    already set on their engines), halo exchanges between hops, then the merged global top-k.
    Returns (ids int64 [B, k] global vertex ids (NO_NODE = none), scores f32 [B, k]).
    fixed=True: the exchanges use fixed-capacity peer slots with no host synchronisation; the
    first such pass calibrates the slots over the host-count path (1.5x the largest per-peer
    count seen), and a pass that overflows a slot raises HaloOverflow after growing it (the
    caller sets seeds / sources again and re-runs -- run_partitioned_retry does that -- and the
    re-run recalibrates).
    overlap (default: on for device engines): the propagation chain (hop, score exchange, hop,
    ...) and the reach chain (reach hop, reach exchange, ...) share no buffer until the top-k, so
    the reach chain runs on a second stream beside it and its hops and exchanges hide under the
    score chain's."""
    # (the fixed-slot kernels map rows of up to 4096 columns; wider plans keep the host counts)
    use_fixed = fixed and sparse and all(r.cap for r in runs) and \
        all(hasattr(r.eng, "pack_sparse_cap") and r.Bpad <= 4096 for r in runs)
    for r in runs:
        r.overflow.zero_()
        if fixed and sparse and not use_fixed:
            r.max_seen = {}
    if overlap is None:
        overlap = all(getattr(r.send, "is_cuda", False) for r in runs)
    dev = runs[0].send.device if runs else None
    main = torch.cuda.current_stream(dev) if overlap else None
    side = _side_stream(dev) if overlap else None
    if overlap:
        side.wait_stream(main)                   # seeds and sources were set on the main stream
    xch = _exchange_fixed if use_fixed else _exchange_sparse if sparse else _exchange
    for h in range(hops):
        for r in runs:
            r.eng.hop()
        if h + 1 < hops:
            xch(runs, comm, "scores")
        with (torch.cuda.stream(side) if overlap else contextlib.nullcontext()):
            for r in runs:
                r.eng.reach_hop()
            if h + 1 < hops:
                xch(runs, comm, "reach")
    if overlap:
        main.wait_stream(side)
    if fixed and sparse and not use_fixed:
        # calibration: the slots hold 1.5x the largest per-peer entry count of this pass (the
        # same on every rank: the all-to-all needs equal block sizes)
        for what in ("scores", "reach"):
            m = max((r.max_seen.get(what, 0) for r in runs), default=0)
            m = _max_over_ranks(comm, m)
            for r in runs:
                r.cap[what] = max(1024, (3 * m) // 2 + 1)
    # the candidate lists travel in one all-gather, each rank's with its overflow flag as a last
    # element: every rank learns whether any slot of the pass overflowed without an all-reduce
    cands = []
    shape = None
    for r in runs:
        r.eng.candidates(exclude_label)
        ids, sc = r.eng.topk(exclude_label)
        lid = ids.to(torch.int64) & 0xFFFFFFFF
        g = torch.where(lid == NO_NODE, torch.full_like(lid, NO_NODE),
                        r.gid[torch.clamp(lid, max=len(r.lg.gid) - 1)])
        c = torch.stack([g.to(torch.float64), sc.to(torch.float64)], dim=0)
        shape = c.shape
        cands.append(torch.cat([c.reshape(-1), r.overflow.to(torch.float64).reshape(1)]))
    gathered = comm.all_gather(cands)
    if use_fixed:
        flags = gathered[0].view(-1, cands[0].numel())[:, -1]
        if bool((flags != 0).any().item()):
            for r in runs:
                r.cap = {}                # the re-run calibrates again over the host counts
                r.overflows += 1
            raise HaloOverflow("a halo exchange overflowed its fixed peer slots (run again)")
    out = []
    for r, allc in zip(runs, gathered):
        allc = allc.view(-1, cands[0].numel())[:, :-1].reshape(-1, *shape[1:])
        P = allc.shape[0] // 2
        ids = allc.view(P, 2, *shape[1:])[:, 0].permute(1, 0, 2).reshape(shape[1], -1)
        scs = allc.view(P, 2, *shape[1:])[:, 1].permute(1, 0, 2).reshape(shape[1], -1)
        # (score desc, id asc): stable sort by id, then stable sort by -score
        o1 = torch.argsort(ids, dim=1, stable=True)
        ids, scs = torch.gather(ids, 1, o1), torch.gather(scs, 1, o1)
        o2 = torch.argsort(-scs, dim=1, stable=True)
        ids, scs = torch.gather(ids, 1, o2)[:, :k], torch.gather(scs, 1, o2)[:, :k]
        out.append((ids.to(torch.int64), scs.to(torch.float32)))
    return out


def _max_over_ranks(comm, x: int) -> int:
    """max of an int over the process group (LocalComm: the value itself -- every local rank
    is already in `runs`)."""
    if not hasattr(comm, "dist"):
        return int(x)
    t = torch.tensor([int(x)], dtype=torch.int64)
    if not comm.gloo:
        import torch as _t
        t = t.to(_t.device("cuda", _t.cuda.current_device()))
    comm.dist.all_reduce(t, op=comm.dist.ReduceOp.MAX, group=comm.group)
    return int(t.item())


def run_partitioned_retry(runs: list[RankRun], comm, hops: int, exclude_label: int, k: int,
                          reset, fixed: bool = True, overlap: bool | None = None):
    """run_partitioned with fixed-capacity slots, re-running once (after `reset()`, which sets
    every engine's seeds and sources again) when a slot overflowed: the re-run goes over the
    host-count path, which cannot overflow, and recalibrates the slots."""
    try:
        return run_partitioned(runs, comm, hops, exclude_label, k, sparse=True, fixed=fixed,
                               overlap=overlap)
    except HaloOverflow:
        reset()
        return run_partitioned(runs, comm, hops, exclude_label, k, sparse=True, fixed=fixed,
                               overlap=overlap)
