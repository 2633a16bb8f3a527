"""How much CSR-row work columns could share (VERDICT r03 item 3's first measurement; CPU only).

For each incident column of a distinct C3 batch: the vertices whose rows a 3-hop pull reads
(hop h pulls the rows of the members within h+1 hops of the seeds; the entries pulled are their
degrees).  For groups of g columns (consecutive after sorting by namespace, by deployment, or
in batch order) the ratio  union of pulled entries / sum of pulled entries  is the fraction of
row loads a column-group pull (one row load feeding g columns) would still issue."""
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "kubernetes-aiops-evidence-graph_amd"))
from egraph import synth  # noqa: E402

B, hops = int(sys.argv[1]) if len(sys.argv) > 1 else 1024, 3
c = synth.build_cluster(synth.CONFIGS["C3"])
cases = synth.make_incidents(c, B, seed=1000)
synth.add_incidents(c, cases)
g = synth.build_graph(c)
csr = g.csr()
rp, col = csr["row_ptr"].astype(np.int64), csr["col"].astype(np.int64)
V = len(rp) - 1
deg = np.diff(rp)
sv, sc, ss = synth.seeds_for_batch(g, [x.evidence for x in cases])


def layers(seeds):
    """rings: members within 1..hops hops of the seeds (as boolean masks, cumulative)"""
    cur = np.zeros(V, bool)
    cur[seeds] = True
    out = []
    for _ in range(hops):
        idx = np.flatnonzero(cur)
        nb = np.concatenate([col[rp[v]:rp[v + 1]] for v in idx]) if len(idx) else np.zeros(0, np.int64)
        nxt = cur.copy()
        nxt[nb] = True
        out.append(nxt)
        cur = nxt
    return out


mem = []
for b in range(B):
    s = np.unique(sv[sc == b].astype(np.int64))
    # pull h reads the rows of the members within h+1 hops (the last pull: within `hops`)
    mem.append([np.flatnonzero(m) for m in layers(s)])
cost = np.array([sum(int(deg[m].sum()) for m in ms) for ms in mem])
ns = np.array([x.incident["namespace"] for x in cases])
dep = np.array([x.incident["service"] for x in cases])
print(f"C3, B={B}: pulled entries per column mean {cost.mean():.0f}, members (3 hops) mean "
      f"{np.mean([len(ms[-1]) for ms in mem]):.0f}; namespaces in batch {len(set(ns))}, "
      f"deployments {len(set(dep))}")
for name, key in (("batch order", np.arange(B)), ("namespace", ns), ("deployment", dep)):
    order = np.argsort(key, kind="stable")
    row = []
    for gsz in (2, 4, 8, 16):
        uni = tot = 0
        for i in range(0, B - B % gsz, gsz):
            grp = order[i:i + gsz]
            tot += int(cost[grp].sum())
            for h in range(hops):
                u = np.unique(np.concatenate([mem[b][h] for b in grp]))
                uni += int(deg[u].sum())
        row.append(f"g={gsz}: {uni / tot:.3f}")
    print(f"  grouped by {name:11s} union/sum  " + "  ".join(row))
