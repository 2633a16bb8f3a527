"""Print one step's kernel timeline (start offset, duration, queue) from a rocprofv3
--kernel-trace CSV of bench.py (diagnostic).  Usage: python timeline.py <csv> [step]"""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
starts = [i for i, r in enumerate(rows) if "rules_eval_kernel" in r["Kernel_Name"]]
k = int(sys.argv[2]) if len(sys.argv) > 2 else -3
a, b = starts[k], starts[k + 1]
t0 = int(rows[a]["Start_Timestamp"])
q = "Queue_Id" if "Queue_Id" in rows[0] else ("Stream_Id" if "Stream_Id" in rows[0] else None)
for r in rows[a - 4:b + 1]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    name = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0][-50:]
    print(f"{(s - t0) / 1e3:9.1f} {(e - s) / 1e3:8.1f}  q={r.get(q, '?') if q else '?':>3}  {name}")
