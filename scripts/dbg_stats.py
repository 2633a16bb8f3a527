import sys, torch
sys.path.insert(0, "kubernetes-aiops-evidence-graph_amd"); sys.path.insert(0, ".")
import bench
dev = torch.device("cuda", 0)
ctx = bench.setup("C3", 1024, 10, 0, dev, pool_entries=-1, merge=20)
fr = ctx["lanes"][0]["frontier"]
bench.step_frontier(ctx, 3)
torch.cuda.synchronize()
print("stats", fr.stats(), flush=True)
