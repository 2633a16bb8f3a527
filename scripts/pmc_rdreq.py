"""Bytes fetched past L2 per frontier_lds_kernel launch from a TCC_EA0_RDREQ / WRREQ counter
pass (rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum -- bench.py):
RDREQ x 128 B (one request per 128-B line for this kernel's 8-B gathers, calibrated by
scripts/calib_gather.hip, profiles/r02_calib_gather.txt) + 32 B per write request (64 B for the
64-B ones).  Writes profiles/pmc_frontier_calibrated_<tag>.json, which bench.py reads when its
workload (config, batch, batches per launch) matches.
Usage: python scripts/pmc_rdreq.py <pmc dir> <tag> <config> <batch> <batches_per_launch> [distinct]
(distinct = how many different incident sets the launch's batches are; 1 = copies of one set)"""
import csv
import hashlib
import json
import os
import sys
from collections import defaultdict
from pathlib import Path

root, tag, config, batch, merge = Path(sys.argv[1]), sys.argv[2], sys.argv[3], int(sys.argv[4]), int(sys.argv[5])
distinct = int(sys.argv[6]) if len(sys.argv) > 6 else 1
REPO = Path(__file__).resolve().parents[1]
LIB = Path(os.environ.get("EGRAPH_LIB", REPO / "kubernetes-aiops-evidence-graph_amd" / "lib" / "libegraph.so"))
vals = defaultdict(list)
for f in sorted(root.rglob("*counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        if "frontier_lds_kernel" in r.get("Kernel_Name", ""):
            vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
mean = {c: sum(x) / len(x) for c, x in vals.items()}
rd, wr, wr64 = mean["TCC_EA0_RDREQ_sum"], mean["TCC_EA0_WRREQ_sum"], mean.get("TCC_EA0_WRREQ_64B_sum", 0.0)
rep = {
    "kernel": "frontier_lds_kernel, %s, %d columns per launch (%d batches of %d, %d different "
              "incident sets), pruned top-10" % (config, batch * merge, merge, batch, distinct),
    "workload": {"config": config, "batch": batch, "batches_per_launch": merge,
                 "distinct_batches": distinct,
                 # the snapshot's locality layout, as bench.frontier_layout_on() reads it
                 "layout": not os.environ.get("EGRAPH_FRONTIER_LAYOUT", "1").startswith("0")},
    "l2_read_requests_per_batch": rd / merge,
    "dispatches": len(vals["TCC_EA0_RDREQ_sum"]),
    "tcc_ea0_rdreq_per_launch": rd, "tcc_ea0_wrreq_per_launch": wr, "tcc_ea0_wrreq_64b_per_launch": wr64,
    "bytes_per_rdreq": 128,
    "read_bytes_per_launch": rd * 128.0,
    "write_bytes_per_launch": wr * 32.0 + wr64 * 32.0,
    "hbm_bytes_per_launch": rd * 128.0 + wr * 32.0 + wr64 * 32.0,
    "note": "bytes fetched past the XCD L2s: Infinity-Cache hits are counted (the 12-MB C3 CSR "
            "is Infinity-Cache resident), so this is an upper bound on HBM bytes",
    "source": str(root),
    # the build the counters were taken on (egraph._lib.build_hash): bench.py reports this file's
    # bytes as roofline.traffic only while it loads the same libegraph.so
    "lib_hash": hashlib.sha256(LIB.read_bytes()).hexdigest()[:16],
}
(REPO / "profiles" / f"pmc_frontier_calibrated_{tag}.json").write_text(json.dumps(rep, indent=1))
print(json.dumps(rep))
