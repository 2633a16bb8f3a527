"""A model of the dense hop's gather re-reads (CPU only): rows are swept in 128-row chunks, chunk i
on XCD i % 8 (the hardware's round-robin) or XCD-contiguous runs of chunks, and each XCD keeps an
LRU of 8,192 neighbour row-tiles (its 4-MB L2 / 512 B).  Misses per vertex are the model's
L2->memory fetches of x per tile sweep (1.0 = every row-tile fetched once, the algorithmic
bytes).  Orders: vertex id (namespace-contiguous), the frontier's hub-forest locality order,
reverse Cuthill-McKee.  Output: profiles/r04_hop_l2_model.txt."""
import sys
from collections import OrderedDict
from pathlib import Path

import numpy as np
import scipy.sparse as sp
from scipy.sparse.csgraph import reverse_cuthill_mckee

sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "kubernetes-aiops-evidence-graph_amd"))
from egraph import synth  # noqa: E402
from egraph.graph import locality_order  # noqa: E402

c = synth.build_cluster(synth.CONFIGS["C3"])
g = synth.build_graph(c)
csr = g.csr()
rp, col = csr["row_ptr"].astype(np.int64), csr["col"].astype(np.int64)
V = len(rp) - 1
ROWS, NX, CAP = 128, 8, 8192


def misses(order, contiguous):
    nch = (V + ROWS - 1) // ROWS
    per = (nch + NX - 1) // NX
    caches = [OrderedDict() for _ in range(NX)]
    m = 0
    seq = sorted(range(nch), key=lambda ci: (ci // per, ci)) if contiguous else range(nch)
    for ci in seq:
        cache = caches[ci // per if contiguous else ci % NX]
        for v in order[ci * ROWS:(ci + 1) * ROWS].tolist():
            for u in col[rp[v]:rp[v + 1]].tolist():
                if u in cache:
                    cache.move_to_end(u)
                else:
                    m += 1
                    cache[u] = 1
                    if len(cache) > CAP:
                        cache.popitem(last=False)
    return m / V


A = sp.csr_matrix((np.ones(len(col)), col, rp), shape=(V, V))
A = ((A + A.T) > 0).astype(np.int8).tocsr()
orders = {"vertex id": np.arange(V), "hub-forest locality": np.asarray(locality_order(csr["row_ptr"], csr["col"])),
          "reverse Cuthill-McKee": np.asarray(reverse_cuthill_mckee(A, symmetric_mode=True))}
print(f"C3: V = {V}, CSR entries = {len(col)}; fetches of x per vertex per tile sweep (model)")
for name, o in orders.items():
    print(f"  {name:22s} round-robin XCDs {misses(o, False):.3f}   XCD-contiguous runs {misses(o, True):.3f}")
