#!/usr/bin/env python3
"""How many of the dense hop's tile gathers read an all-zero tile?  (CPU, the host CSR.)
Per column the non-zero rows after hop h are at most the vertices within h hops of its seeds
(boolean sparse products); a (vertex, tile) of TW columns is non-zero if any of its columns is.
The hop gathers x[u][tile] once per CSR entry (v -> u) per tile: the fraction of those gathers
whose tile is all-zero is what a per-tile non-zero flag lets the hop skip (fmaf(w, +0, acc) ==
acc: exact).  Usage: python scripts/tile_sparsity.py C3|C4 [B] [TW]"""
import sys, time
import numpy as np
import scipy.sparse as sp
sys.path.insert(0, "kubernetes-aiops-evidence-graph_amd")
from egraph import synth

cfg = sys.argv[1] if len(sys.argv) > 1 else "C3"
B = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
TW = int(sys.argv[3]) if len(sys.argv) > 3 else 128
t0 = time.time()
cl = synth.build_cluster(synth.CONFIGS[cfg])
cases = synth.make_incidents(cl, B, seed=1000)
synth.add_incidents(cl, cases)
g = synth.build_graph(cl)
csr = g.csr()
V = g.num_vertices
sv, sc, ss = synth.seeds_for_batch(g, [x.evidence for x in cases])
rp = csr["row_ptr"].astype(np.int64)
A = sp.csr_matrix((np.ones(len(csr["col"]), np.float32), csr["col"].astype(np.int64), rp), shape=(V, V))
X = sp.csr_matrix((np.ones(len(sv), np.float32), (sv.astype(np.int64), sc.astype(np.int64))), shape=(V, B))
X.data[:] = 1
indeg = np.bincount(csr["col"].astype(np.int64), minlength=V).astype(np.float64)   # gathers per vertex
ntiles = (B + TW - 1) // TW
print(f"{cfg}: V={V} entries={len(csr['col'])} B={B} TW={TW} ({time.time()-t0:.1f}s)")
for h in range(1, 4):
    # x_h non-zero pattern: seeds (s0 is added every hop) plus A x_{h-1}
    X = (A @ X + X).tocsr()
    X.data[:] = 1
    Xc = X.tocoo()
    tiles = sp.csr_matrix((np.ones(Xc.nnz, np.float32), (Xc.row, Xc.col // TW)), shape=(V, ntiles))
    tiles.sum_duplicates()
    nzt = np.asarray((tiles > 0).sum(axis=1)).ravel()           # non-zero tiles per vertex
    frac_gathers = float((indeg * nzt).sum() / (indeg.sum() * ntiles))
    print(f"x after hop {h}: non-zero entries {X.nnz / (V * B):.4%} of V x B; non-zero tiles "
          f"{nzt.sum() / (V * ntiles):.2%} of (vertex, tile); gathers of hop {h + 1} on non-zero tiles "
          f"{frac_gathers:.2%}")
