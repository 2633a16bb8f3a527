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
Exports of r = owned vertices with a neighbour owned elsewhere.

Per hop (RankRun.run): the engine computes its rows; the owners' fresh export rows are packed,
all-gathered (RCCL over xGMI: torch.distributed all_gather_into_tensor on device buffers,
[P * max_export][Bpad] fp32 for scores and [..][ceil(B/64)] u64 for reach) and unpacked into the
halo rows.  After the last hop each rank ranks its owned candidates; the (score, global id)
lists are all-gathered and merged (score desc, global id asc) -- the unpartitioned top-k.
Scores, reach sets and top-k are bit-identical to the single-GPU plan (tests/test_shard*.py).
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np
import torch

NO_NODE = 0xFFFFFFFF


def partition_vertices(row_ptr: np.ndarray, vlabel: np.ndarray, label_names: list[str], P: int,
                       hash_labels: tuple[str, ...] = ("Node",)) -> np.ndarray:
    """owner[v] in [0, P): hashed for `hash_labels`, entry-balanced contiguous ranges otherwise."""
    V = len(row_ptr) - 1
    if P < 1:
        raise ValueError("P must be >= 1")
    owner = np.zeros(V, np.int32)
    if P == 1:
        return owner
    hashed = np.isin(vlabel, [label_names.index(n) for n in hash_labels if n in label_names])
    deg = np.diff(row_ptr.astype(np.int64))
    w = np.where(hashed, 0, deg + 1)            # +1: isolated vertices still weigh something
    cum = np.cumsum(w)
    total = int(cum[-1]) if V else 0
    owner[:] = np.minimum((cum - 1) * P // max(total, 1), P - 1).astype(np.int32)
    ids = np.flatnonzero(hashed).astype(np.uint64)
    owner[hashed] = ((ids * np.uint64(0x9E3779B1)) >> np.uint64(7)) % np.uint64(P)
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
    export_rows: np.ndarray  # local ids (owned) this rank sends, in global order
    halo_rows: np.ndarray    # local ids of the halo rows
    halo_src: np.ndarray     # per halo row: index into the all-gathered export rows
    max_export: int


def build_local(csr: dict, vlabel: np.ndarray, owner: np.ndarray, rank: int, P: int) -> LocalGraph:
    """Rank `rank`'s local CSR and exchange maps from the global host CSR (graph.csr())."""
    rp = csr["row_ptr"].astype(np.int64)
    col = csr["col"].astype(np.int64)
    V = len(rp) - 1
    deg = np.diff(rp)
    src_of = np.repeat(np.arange(V, dtype=np.int64), deg)
    cross = owner[src_of] != owner[col]         # entry (v -> u) across ranks: u is v's halo
    # exports of every rank (all ranks compute all of them: max_export must agree)
    exp_mask = np.zeros(V, bool)
    exp_mask[col[cross]] = True                 # u has a neighbour owned elsewhere
    exports = [np.flatnonzero(exp_mask & (owner == r)) for r in range(P)]
    max_export = max([len(e) for e in exports] + [1])
    owned = np.flatnonzero(owner == rank)
    mine = owner[src_of] == rank
    halo = np.unique(col[mine & cross])
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
    pos_in_export = np.full(V, -1, np.int64)
    for r in range(P):
        pos_in_export[exports[r]] = np.arange(len(exports[r]))
    halo_src = owner[halo].astype(np.int64) * max_export + pos_in_export[halo]
    assert (pos_in_export[halo] >= 0).all()
    return LocalGraph(
        rank=rank, P=P, gid=gid, n_owned=len(owned),
        row_ptr=l_rp.astype(np.uint32), col=g2l[col[take]].astype(np.uint32),
        meta=csr["meta"][take].astype(np.uint8), val=csr["val"][take].astype(np.float32),
        vlabel=vlabel[gid].astype(np.uint8),
        export_rows=g2l[exports[rank]].astype(np.uint32),
        halo_rows=np.arange(len(owned), len(gid), dtype=np.uint32),
        halo_src=halo_src.astype(np.uint32), max_export=max_export)


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
    """All-gather across the process group: RCCL all_gather_into_tensor on device buffers (the
    production path, one process per GPU); under gloo (CPU tests, or several processes sharing
    one GPU, which RCCL refuses) the buffers are staged through host memory."""

    def __init__(self, group=None):
        import torch.distributed as dist
        self.dist = dist
        self.group = group
        self.P = dist.get_world_size(group)
        self.gloo = dist.get_backend(group) == "gloo"

    def all_gather(self, send: list[torch.Tensor]) -> list[torch.Tensor]:
        (x,) = send
        x = x.contiguous()
        if self.gloo:
            h = x.cpu()
            parts = [torch.empty_like(h) for _ in range(self.P)]
            self.dist.all_gather(parts, h, group=self.group)
            return [torch.cat(parts).to(x.device)]
        out = torch.empty((self.P * x.shape[0],) + tuple(x.shape[1:]), dtype=x.dtype, device=x.device)
        self.dist.all_gather_into_tensor(out, x, group=self.group)
        return [out]


class LocalComm:
    """All ranks in one process (tests, and a multi-partition single-GPU run): the gather is a
    concatenation of the ranks' buffers."""

    def all_gather(self, send: list[torch.Tensor]) -> list[torch.Tensor]:
        cat = torch.cat([s.to(send[0].device) for s in send])
        return [cat.to(s.device) for s in send]


class RankRun:
    """One rank's part of a partitioned pass.  `engine` is the HIP Plan of the local snapshot
    (egraph.graph.Plan); any object with the same methods works (the CPU tests use the oracle)."""

    def __init__(self, lg: LocalGraph, engine, device):
        self.lg, self.eng, self.dev = lg, engine, device
        self.exp = torch.from_numpy(lg.export_rows.view(np.int32)).to(device)
        self.halo = torch.from_numpy(lg.halo_rows.view(np.int32)).to(device)
        self.src = torch.from_numpy(lg.halo_src.view(np.int32)).to(device)
        self.gid = torch.from_numpy(lg.gid).to(device)
        B = engine.B
        self.Bpad = engine.padded_cols
        self.W = (B + 63) // 64
        self.send_s = torch.zeros((lg.max_export, self.Bpad), dtype=torch.float32, device=device)
        self.send_r = torch.zeros((lg.max_export, self.W), dtype=torch.int64, device=device)
        engine.set_owned(lg.n_owned)


def _exchange(runs: list[RankRun], comm, what: str) -> None:
    sends = []
    for r in runs:
        buf = r.send_s if what == "scores" else r.send_r
        (r.eng.pack_scores if what == "scores" else r.eng.pack_reach)(r.exp, buf)
        sends.append(buf)
    recvs = comm.all_gather(sends)
    for r, rv in zip(runs, recvs):
        (r.eng.unpack_scores if what == "scores" else r.eng.unpack_reach)(r.halo, r.src, rv)


def run_partitioned(runs: list[RankRun], comm, hops: int, exclude_label: int, k: int):
    """`hops` hops of propagation and reach on every local rank in `runs` (seeds and sources
    already set on their engines), halo exchanges between hops, then the merged global top-k.
    Returns (ids int64 [B, k] global vertex ids (NO_NODE = none), scores f32 [B, k])."""
    for h in range(hops):
        for r in runs:
            r.eng.hop()
        if h + 1 < hops:
            _exchange(runs, comm, "scores")
        for r in runs:
            r.eng.reach_hop()
        if h + 1 < hops:
            _exchange(runs, comm, "reach")
    cands = []
    for r in runs:
        r.eng.candidates(exclude_label)
        ids, sc = r.eng.topk(exclude_label)
        lid = ids.to(torch.int64) & 0xFFFFFFFF
        g = torch.where(lid == NO_NODE, torch.full_like(lid, NO_NODE),
                        r.gid[torch.clamp(lid, max=len(r.lg.gid) - 1)])
        cands.append(torch.stack([g.to(torch.float64), sc.to(torch.float64)], dim=0))
    gathered = comm.all_gather(cands)
    out = []
    for r, allc in zip(runs, gathered):
        P = allc.shape[0] // 2
        ids = allc.view(P, 2, *cands[0].shape[1:])[:, 0].permute(1, 0, 2).reshape(cands[0].shape[1], -1)
        scs = allc.view(P, 2, *cands[0].shape[1:])[:, 1].permute(1, 0, 2).reshape(cands[0].shape[1], -1)
        # (score desc, id asc): stable sort by id, then stable sort by -score
        o1 = torch.argsort(ids, dim=1, stable=True)
        ids, scs = torch.gather(ids, 1, o1), torch.gather(scs, 1, o1)
        o2 = torch.argsort(-scs, dim=1, stable=True)
        ids, scs = torch.gather(ids, 1, o2)[:, :k], torch.gather(scs, 1, o2)[:, :k]
        out.append((ids.to(torch.int64), scs.to(torch.float32)))
    return out
