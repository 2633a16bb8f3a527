"""Per-phase wall time of the local frontier kernel (csrc/frontier_local.h) on a bench batch (GPU).

Creates a top-k-only frontier with $EGRAPH_FRONTIER_PROFILE set, runs one C3 batch a few
times and prints the mean / p50 / p99 per-column duration of each phase from the kernel's
s_memrealtime stamps (100 MHz): seeds, expansion walks 1..H, the local-CSR walk, propagation +
top-k."""
import os
import sys
from pathlib import Path

import numpy as np

os.environ["EGRAPH_FRONTIER_PROFILE"] = "1"
REPO = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(REPO), str(REPO / "kubernetes-aiops-evidence-graph_amd")]
import torch  # noqa: E402

import bench  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "C3"
B = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
H = 3
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
ctx = bench.setup(cfg, B, 10, 0, dev, pipeline=1, pool_entries=-1)
fr = ctx["frontier"]
lane = ctx["lanes"][0]
for _ in range(5):
    fr.set_seeds(*lane["seeds"])
    fr.run(lane["sources"], H, ctx["inc_label"])
torch.cuda.synchronize()
t = fr.phase_times()[:, :, 0].astype(np.int64)          # [B, 40] post-barrier stamps, thread 0
names = ["seeds"] + [f"walk{k}" for k in range(1, H + 1)] + ["local_csr"] + \
    [f"hop{h}" for h in range(H)] + ["topk"]
print(f"{cfg} B={B}: per-column phase times (us), mean / p50 / p99")
last = 3 + 2 * H
tot = (t[:, last] - t[:, 0]) / 100.0
for i, n in enumerate(names):
    d = (t[:, i + 1] - t[:, i]) / 100.0
    print(f"  {n:16s} {d.mean():8.2f} {np.percentile(d, 50):8.2f} {np.percentile(d, 99):8.2f}")
print(f"  {'column':16s} {tot.mean():8.2f} {np.percentile(tot, 50):8.2f} {np.percentile(tot, 99):8.2f}")
start = (t[:, 0] - t[:, 0].min()) / 100.0
end = (t[:, last] - t[:, 0].min()) / 100.0
print(f"  columns start over {start.max():.1f} us, last ends at {end.max():.1f} us")
ec, nm = t[:, 30], t[:, 31]
prop = (t[:, last] - t[:, 2 + H]) / 100.0
print(f"  local entries mean {ec.mean():.0f} max {ec.max()}, members mean {nm.mean():.0f} max {nm.max()}")
for lo, hi in ((0, 1000), (1000, 1400), (1400, 1848), (1848, 1 << 20)):
    m = (ec >= lo) & (ec < hi)
    if m.any():
        print(f"  entries [{lo},{hi}): {m.sum()} columns, propagate+topk mean {prop[m].mean():.1f} us")
print("stats", fr.stats())
