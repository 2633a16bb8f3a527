#!/bin/bash
# A/B of the default libegraph.so build against variant builds on the bench, interleaved on one
# box: for each of REPS rounds, the default build then each variant in $ALTS (paths relative to
# the repo, built by scripts/build_variant.sh).  Optional parity first: TESTS (pytest node ids)
# run against every variant.  Env: TAG (output dir), ALTS, REPS (default 3), BENCH_ARGS (default:
# the driver's --steps 20 --warmup 5 without the host-side extras), ENV_ALTS (alternatives of the
# default build under an environment setting: "name:VAR=value ...").
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-ab}
mkdir -p $OUT
ARGS=${BENCH_ARGS:-"--steps 20 --warmup 5 --no-cpu-baseline --no-dropin --dense-steps 0 --roofline-reps 5"}
if [ -n "$TESTS" ]; then          # (parity of the default build, the candidate)
  timeout -k 10 400 python -u -m pytest $TESTS -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1
  echo "tests ok: $(tail -1 $OUT/pytest.log)"
  if [ -n "$VARIANT_TESTS" ]; then  # (and of every variant build)
    for a in $ALTS; do
      n=$(basename $(dirname $a))
      EGRAPH_LIB=$PWD/$a timeout -k 10 400 python -u -m pytest $TESTS -x -q --timeout 200 --timeout-method thread > $OUT/pytest_$n.log 2>&1
      echo "tests ok ($n): $(tail -1 $OUT/pytest_$n.log)"
    done
  fi
fi
for r in $(seq 1 ${REPS:-3}); do
  for a in base $ALTS $ENV_ALTS; do
    ev=""
    if [ $a = base ]; then unset EGRAPH_LIB; n=base
    elif [[ $a == *:* ]]; then unset EGRAPH_LIB; n=${a%%:*}; ev=${a#*:}
    else export EGRAPH_LIB=$PWD/$a; n=$(basename $(dirname $a)); fi
    env $ev timeout -k 10 200 python bench.py $ARGS > $OUT/${n}_$r.json 2> $OUT/${n}_$r.err
    python -c "import json;d=json.load(open('$OUT/${n}_$r.json'));r=d['roofline'];w=d.get('frontier_work',{});print('$n', $r, round(d['value']), round(d['ms_per_step'],5), 'launch', round(r['avg_launch_ms'],4), 'ovf', w.get('overflowed'), 'cont', w.get('continued'))"
  done
done
