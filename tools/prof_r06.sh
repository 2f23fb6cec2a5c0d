#!/bin/bash
# Round-6 profile pass on the GPU box: front kernel PMC at the headline preset
# (e7) and at effort 4 (the literal fused XYB + DCT + quant of SURVEY 8(d)),
# merge_eval PMC, and a kernel trace of a short default bench.
# Usage: bash tools/prof_r06.sh TAG [front|e4|merge|trace ...]
set -e
export TMPDIR=/tmp
TAG=${1:-r06p}; shift || true
STEPS=${@:-front e4 merge trace}
O=gpurun_out/$TAG
mkdir -p $O
B="--steps 2 --warmup 1 --no-cpu-baseline --no-quality --no-single --alt-coder 0 --alt-thesis 0 --alt-cjxl 0 --alt-e4 0 --no-pipeline"
for s in $STEPS; do
  case $s in
    front) EXTRA=1 bash profiles/pmc_front.sh $O/pmc_front ;;
    e4) EXTRA=1 BENCH_ARGS="$B --effort 4" bash profiles/pmc_front.sh $O/pmc_e4 ;;
    merge) KERNEL=merge_eval_kernel bash profiles/pmc_front.sh $O/pmc_merge ;;
    trace) timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $PWD/$O/prof -o run -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-quality --no-single > $O/bench_prof.log 2>&1 ;;
  esac
done
