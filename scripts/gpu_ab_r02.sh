set -e
TAG=abm1 LIBS="default exp_lsnew1536 exp_ft128 exp_lcap1536" REPS="1 2" STEPS=200 bash scripts/ab_multi.sh
mkdir -p gpurun_out/abm1x
for r in 1 2; do EGRAPH_FRONTIER_XCD=1 timeout -k 10 200 python bench.py --no-cpu-baseline --no-dropin --dense-steps 0 --steps 200 > gpurun_out/abm1x/xcd$r.json 2>gpurun_out/abm1x/xcd$r.err; python -c "import json;d=json.load(open('gpurun_out/abm1x/xcd$r.json'));print('xcd', d['value'], d['ms_per_step'])"; done
TAG=pmcf1 bash scripts/pmc_frontier_r02.sh
