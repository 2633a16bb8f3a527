"""The frontier engine's global-memory fallback (frontier_global_kernel) on large graphs.

Columns that overflow the LDS tables are redone with a table in HBM; these cases push many
columns of a 100k-pod (C3-sized) graph, and columns of a 240k-vertex star, through it and
compare with the C oracle (oracle/egraph_oracle.c)."""
from __future__ import annotations

import numpy as np
import pytest

from test_frontier_gpu import _check, _hub_world

pytestmark = pytest.mark.gpu


def test_fallback_large_star():
    g, sv, sc, ss, src = _hub_world(n_leaves=120_000, n_cols=4)
    fr = _check(g, sv, sc, ss, src, len(src), k=10, pool_entries=-1, scores=False)
    assert fr.stats()["overflowed"] >= 2


def test_fallback_c3_columns(monkeypatch):
    """Every column of a C3 batch through the global-memory variant
    ($EGRAPH_FRONTIER_GLOBAL_ONLY: as if the LDS kernels had handed every column on), pruned and
    with a member pool."""
    from egraph import synth
    from egraph.graph import EvidenceGraph
    monkeypatch.setenv("EGRAPH_FRONTIER_GLOBAL_ONLY", "1")
    B = 48
    c = synth.build_cluster(synth.CONFIGS["C3"])
    cases = synth.make_incidents(c, B, seed=1000)
    synth.add_incidents(c, cases)
    g = EvidenceGraph()
    g.merge_nodes(c.ids, c.labels)
    g.merge_edges(c.src, c.dst, c.types)
    sv, sc, ss = synth.seeds_for_batch(g, [x.evidence for x in cases])
    src = g.lookup([f"incident:{x.incident['id']}" for x in cases]).astype(np.uint32)
    fr = _check(g, sv, sc, ss, src, B, pool_entries=-1, scores=False)
    assert fr.stats()["members"] > 0
    _check(g, sv, sc, ss, src, B, pool_entries=0, scores=False)
