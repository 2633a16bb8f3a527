"""Distribution of frontier members per incident column on a bench workload (GPU).

Used to size the LDS table: a column with more members than LLIMIT overflows to the
global-memory variant."""
import json
import sys
from pathlib import Path

import numpy as np
import torch

REPO = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(REPO), str(REPO / "kubernetes-aiops-evidence-graph_amd")]
import bench  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "C3"
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
ctx = bench.setup(cfg, 1024, 10, 0, dev)
bench.step_frontier(ctx, 3)
torch.cuda.synchronize()
fr = ctx["frontier"]
n = np.array([len(fr.members(c)[0]) for c in range(fr.B)])
q = np.percentile(n, [0, 10, 50, 90, 99, 99.9, 100])
out = {"config": cfg, "mean": float(n.mean()), "percentiles_0_10_50_90_99_99.9_100": q.tolist(),
       "over": {str(t): int((n > t).sum()) for t in (1536, 2048, 2560, 3072, 3584, 4096, 4608)}}
print(json.dumps(out))
