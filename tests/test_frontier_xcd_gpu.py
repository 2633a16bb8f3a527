"""GPU parity of the opt-in XCD-aware column queues (EGRAPH_FRONTIER_XCD=1, csrc/frontier.hip).

With the switch on, the seed scan queues the columns per graph region and each workgroup pops
the queue of its own XCD (HW_REG_XCC_ID) instead of taking column order[blockIdx].  Placement
may change only speed: the top-k ids and scores must equal the oracle's, for pruned (top-k
only) and member-pool runs, with the largest hub seeded in every column, and on a second run over
the same seeds (the queue heads are reset by the fallback grid).  The switch is read once per
process, so the checks run in one child process with the variable set.
"""
from __future__ import annotations

import os
import subprocess
import sys
from pathlib import Path

import pytest

pytestmark = pytest.mark.gpu

REPO = Path(__file__).resolve().parents[1]

CHILD = r"""
import sys
for p in (sys.argv[1] + "/kubernetes-aiops-evidence-graph_amd", sys.argv[1] + "/oracle",
          sys.argv[1] + "/tests"):
    sys.path.insert(0, p)
import numpy as np
import torch
import test_frontier_gpu as t

torch.cuda.set_device(0)
B = 96
g, sv, sc, ss, src = t._world(B, seed=23)
t._check(g, sv, sc, ss, src, B, pool_entries=-1, scores=False)     # pruned, narrow table
t._check(g, sv, sc, ss, src, B, pool_entries=0)                    # member pool, wide table
# a second run over the same seeds takes its columns from freshly reset queues
fr = g.snapshot().frontier(B, max_seeds=len(sv), k=10, pool_entries=-1)
fr.set_seeds(t._dev(sv), t._dev(sc), t._dev(ss))
inc = g.labels().index("Incident")
a = [x.cpu().numpy().copy() for x in fr.run(t._dev(src), hops=3, exclude_label=inc)]
b = [x.cpu().numpy().copy() for x in fr.run(t._dev(src), hops=3, exclude_label=inc)]
assert all((x.view(np.uint32) == y.view(np.uint32)).all() for x, y in zip(a, b))
# the largest hub seeded in every column: the heaviest columns of this graph
hub = np.full(B, int(np.argmax(np.diff(g.csr()["row_ptr"]))), np.uint32)
t._check(g, np.concatenate([sv, hub]), np.concatenate([sc, np.arange(B, dtype=np.uint32)]),
         np.concatenate([ss, np.full(B, 0.5, np.float32)]), src, B, pool_entries=-1, scores=False)
print("xcd ok")
"""


def test_xcd_queues_match_oracle():
    env = dict(os.environ, EGRAPH_FRONTIER_XCD="1")
    r = subprocess.run([sys.executable, "-c", CHILD, str(REPO)], env=env, capture_output=True,
                       text=True, timeout=110)
    assert r.returncode == 0 and "xcd ok" in r.stdout, r.stdout[-2000:] + r.stderr[-4000:]
