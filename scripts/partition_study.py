#!/usr/bin/env python3
"""Halo / owned of edge-cut partitions of the C4 graph under several ownership rules (CPU; the
host CSR).  halo(r) = the distinct non-r-owned vertices that r-owned rows read; the dense hop
writes owned rows and reads halo tiles, the exchange ships halo rows.
Usage: python scripts/partition_study.py [C4] [P]"""
import sys, time
import numpy as np
sys.path.insert(0, "kubernetes-aiops-evidence-graph_amd")
from egraph import shard, synth

cfg = sys.argv[1] if len(sys.argv) > 1 else "C4"
P = int(sys.argv[2]) if len(sys.argv) > 2 else 8
t0 = time.time()
cl = synth.build_cluster(synth.CONFIGS[cfg])
cases = synth.make_incidents(cl, 1024, seed=1000)
synth.add_incidents(cl, cases)
g = synth.build_graph(cl)
csr = g.csr()
vl, _, _, _ = g.export()
labels = g.labels()
rp = csr["row_ptr"].astype(np.int64)
col = csr["col"].astype(np.int64)
V = len(rp) - 1
deg = np.diff(rp)
src = np.repeat(np.arange(V), deg)
lab = np.array(labels)[vl]
print(f"{cfg}: V={V} entries={len(col)} ({time.time() - t0:.0f}s); labels:",
      {l: int((lab == l).sum()) for l in labels})


def halo_stats(owner, name):
    cross = owner[src] != owner[col]
    pairs = np.unique(owner[src[cross]].astype(np.int64) * V + col[cross])
    reader = pairs // V
    halo = np.bincount(reader, minlength=P)
    owned = np.bincount(owner, minlength=P)
    w = np.bincount(owner, weights=deg + 1, minlength=P)
    print(f"{name:46s} halo/owned max {np.max(halo / owned):.3f} mean {np.mean(halo / owned):.3f}; "
          f"row-weight imbalance max/mean {w.max() / w.mean():.3f}; cut entries {cross.mean():.3f}")
    return halo / owned


base = shard.partition_vertices(csr["row_ptr"], vl, labels, P)
halo_stats(base, "S0: namespace ranges + Node hash (shipped)")
# S1: every Pod and its attachments (Event / LogPattern / MetricAnomaly rows read their pod)
# placed with the pod's Node; the rest by the ranges
is_pod = lab == "Pod"
node_of = np.full(V, -1, np.int64)
sched = (lab[src] == "Pod") & (lab[col] == "Node")
node_of[src[sched]] = col[sched]
s1 = base.copy()
s1[is_pod] = base[node_of[is_pod]]
att = np.isin(lab, ["Event", "LogPattern", "MetricAnomaly"])
pod_of = np.full(V, -1, np.int64)
ap = att[src] & is_pod[col]
pod_of[src[ap]] = col[ap]
ok = att & (pod_of >= 0)
s1[ok] = s1[pod_of[ok]]
halo_stats(s1, "S1: pods + attachments with their Node")
# S2: S1 and each Deployment with the majority of its pods (ties: lowest rank)
dep = lab == "Deployment"
dp = dep[src] & is_pod[col]
cnt = np.zeros((V, P), np.int32)
np.add.at(cnt, (src[dp], s1[col[dp]]), 1)
s2 = s1.copy()
d_idx = np.flatnonzero(dep & (cnt.sum(1) > 0))
s2[d_idx] = np.argmax(cnt[d_idx], axis=1)
halo_stats(s2, "S2: S1 + Deployments with most of their pods")
# S3: Nodes by the namespace-range majority of their pods (a Node's pods span namespaces)
nd = (lab[src] == "Node") & is_pod[col]
cntn = np.zeros((V, P), np.int32)
np.add.at(cntn, (src[nd], base[col[nd]]), 1)
s3 = base.copy()
n_idx = np.flatnonzero((lab == "Node") & (cntn.sum(1) > 0))
s3[n_idx] = np.argmax(cntn[n_idx], axis=1)
halo_stats(s3, "S3: ranges + Nodes with most of their pods")
