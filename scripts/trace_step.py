"""Per-step timeline from a rocprofv3 --kernel-trace CSV of bench.py: kernels, durations and the
idle gaps between consecutive kernels (host/launch overhead).  Usage: python trace_step.py <csv>"""
import csv
import sys
from collections import defaultdict

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
# one step starts at each rules_eval_kernel launch
starts = [i for i, r in enumerate(rows) if "rules_eval_kernel" in r["Kernel_Name"]]
if len(starts) < 3:
    sys.exit("need >= 3 steps in the trace")
acc = defaultdict(float)
gap_total = busy_total = span_total = 0.0
n = 0
for a, b in zip(starts[-6:-1], starts[-5:]):
    steps = rows[a:b]
    t0 = int(steps[0]["Start_Timestamp"])
    t1 = int(rows[b]["Start_Timestamp"])
    span_total += (t1 - t0) / 1e3
    prev_end = t0
    for r in steps:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        name = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0][-60:]
        acc[name] += (e - s) / 1e3
        busy_total += (e - s) / 1e3
        gap_total += max(0, s - prev_end) / 1e3
        prev_end = max(prev_end, e)
    n += 1
print(f"steps {n}: span {span_total / n:.1f} us, kernels {busy_total / n:.1f} us, gaps {gap_total / n:.1f} us")
for k, v in sorted(acc.items(), key=lambda x: -x[1]):
    print(f"  {v / n:8.1f} us  {k}")
