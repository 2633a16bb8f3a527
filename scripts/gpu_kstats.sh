#!/bin/bash
# rocprofv3 kernel stats of the driver's bench line (--steps 20 --warmup 5) under several
# environment settings on ONE box (same-box kernel durations for an A/B).  Env: TAG, RUNS =
# "name:VAR=value[,VAR=value] ..." ("name:" for the defaults), BENCH_ARGS.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-kstats}
mkdir -p $OUT
for run in ${RUNS:-"base:"}; do
  n=${run%%:*}; ev=${run#*:}
  env ${ev//,/ } timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$n -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-dropin --dense-steps 0 ${BENCH_ARGS:-} > $OUT/$n.log 2>&1
  python3 - $OUT/$n <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
print(sys.argv[1].split("/")[-1], "; ".join("%s x%s %.1f us" % (r["Name"].split("(")[1 if r["Name"].startswith("(") else 0].split("::")[-1][:40] if False else r["Name"][:70], r["Calls"], float(r["AverageNs"]) / 1000) for r in rows[:6]))
PY
done
