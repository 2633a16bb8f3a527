"""Per-column shape of the frontier work on a bench workload (CPU, numpy; no GPU).

For each incident column b: S = its seed vertices, src = its incident vertex.
  C      = vertices within `hops` hops of src (the top-k candidates, before the label filter)
  B2     = vertices within hops - 1 hops of S (the only vertices whose s^h, h < hops, can be
           non-zero)
  M      = B2 | C (every vertex whose score the local engine computes)
  rows   = sum of the CSR degrees of M's rows (every member row is read once)
  local  = entries of M's rows whose target is in B2 (the member-restricted local CSR)
  hubs   = member rows longer than 12 entries
Sizes the LDS budget of the two-phase (discover, then propagate over a local CSR) kernel."""
import sys
import time
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(REPO / "kubernetes-aiops-evidence-graph_amd")]
from egraph import synth  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "C3"
B = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
hops = 3
t0 = time.time()
cl = synth.build_cluster(synth.CONFIGS[cfg])
cases = synth.make_incidents(cl, B, seed=1000)
synth.add_incidents(cl, cases)
g = synth.build_graph(cl)
ev = [x.evidence for x in cases]
sv, sc, ss = synth.seeds_for_batch(g, ev)
src = g.lookup([f"incident:{x.incident['id']}" for x in cases]).astype(np.int64)
csr = g.csr()
rp, col = csr["row_ptr"].astype(np.int64), csr["col"].astype(np.int64)
print(f"built {cfg} V={g.num_vertices} nnz={len(col)} in {time.time() - t0:.1f}s", file=sys.stderr)


def ball(start, depth):
    seen = set(int(x) for x in start)
    front = list(seen)
    for _ in range(depth):
        nxt = []
        for v in front:
            for u in col[rp[v]:rp[v + 1]]:
                u = int(u)
                if u not in seen:
                    seen.add(u)
                    nxt.append(u)
        front = nxt
    return seen


order = np.argsort(sc, kind="stable")
bounds = np.searchsorted(sc[order], np.arange(B + 1))
stat = []
for b in range(B):
    S = np.unique(sv[order[bounds[b]:bounds[b + 1]]])
    C = ball([src[b]], hops) if src[b] >= 0 else set()
    B2 = ball(S, hops - 1)
    M = B2 | C
    rows = sum(int(rp[v + 1] - rp[v]) for v in M)
    hubs = sum(1 for v in M if rp[v + 1] - rp[v] > 12)
    hub_e = sum(int(rp[v + 1] - rp[v]) for v in M if rp[v + 1] - rp[v] > 12)
    local = 0
    for v in M:
        for u in col[rp[v]:rp[v + 1]]:
            if int(u) in B2:
                local += 1
    stat.append((len(S), len(C), len(B2), len(M), rows, local, hubs, hub_e))
a = np.array(stat)
names = ["seeds", "C", "B2", "M", "row_entries", "local_entries", "hub_rows", "hub_entries"]
pct = [0, 50, 90, 99, 99.9, 100]
print(f"{cfg} B={B}: per column mean / p0 p50 p90 p99 p99.9 p100")
for i, n in enumerate(names):
    q = np.percentile(a[:, i], pct)
    print(f"  {n:14s} {a[:, i].mean():9.1f}  " + " ".join(f"{x:8.0f}" for x in q))
print(f"  total local entries per batch {a[:, 5].sum()}, row entries {a[:, 4].sum()}, members {a[:, 3].sum()}")
