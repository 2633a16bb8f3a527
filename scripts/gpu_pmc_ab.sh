#!/bin/bash
# Counter A/B: the SQ counter passes of scripts/gpu_pmc.sh over the default build and each
# alternative (ALTS: variant libegraph.so paths; ENV_ALTS: "name:VAR=value ..."), one after the
# other on one box, summarised side by side for the narrow frontier kernel.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-pmcab}
mkdir -p $OUT
for a in base $ALTS $ENV_ALTS; do
  ev=""
  if [ $a = base ]; then unset EGRAPH_LIB; n=base
  elif [[ $a == *:* ]]; then unset EGRAPH_LIB; n=${a%%:*}; ev=${a#*:}
  else export EGRAPH_LIB=$PWD/$a; n=$(basename $(dirname $a)); fi
  for v in $ev; do export "$v"; done
  TAG=${TAG:-pmcab}/$n PASSES="${PASSES:-sq1 sq2}" bash scripts/gpu_pmc.sh > $OUT/$n.txt 2>&1
  for v in $ev; do unset "${v%%=*}"; done
  echo "== $n"; grep -A40 "== frontier_lds_kernel" $OUT/$n/summary.txt | grep -E "SQ_INSTS|SQ_WAVE_CYCLES|SQ_WAIT_ANY|SQ_ACTIVE_INST_VALU|SQ_LDS_BANK|SQ_BUSY" || true
done
