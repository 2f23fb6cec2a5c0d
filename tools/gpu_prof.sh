#!/bin/bash
# Profiles for profiles/: kernel trace + stats of the bench's timed command
# (reduced side lines), the PMC passes of the front kernel and merge_eval
# (profiles/pmc_front.sh, one counter group per pass), the merge tile-chunk
# A/B, the counter list.  Usage: bash tools/gpu_prof.sh TAG [counters] [trace] [pmc] [attr] [chunk] [aq]
export TMPDIR=/tmp
TAG=$1; shift
O=gpurun_out/$TAG
mkdir -p $O
R=$PWD
for s in "$@"; do
  case $s in
    counters) timeout -k 10 120 rocprofv3 -L > $O/counters.txt 2>&1 || exit $? ;;
    trace) timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/trace -o run -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-quality --alt-coder 0 --alt-thesis 0 --alt-cjxl 0 > $O/trace_bench.log 2>&1 || exit $? ;;
    pmc) bash profiles/pmc_front.sh $O/pmc_front || exit $?
         KERNEL=merge_eval_kernel bash profiles/pmc_front.sh $O/pmc_merge || exit $? ;;
    attr) EXTRA=1 KERNEL=merge_eval_kernel bash profiles/pmc_front.sh $O/attr_merge || exit $?
          EXTRA=1 bash profiles/pmc_front.sh $O/attr_front || exit $? ;;
    chunk) bash tools/merge_chunk_ab.sh run $TAG || exit $? ;;
    aq) timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/trace_cjxl -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-quality --alt-coder 0 --alt-thesis 0 --alt-cjxl 1 > $O/trace_cjxl.log 2>&1 || exit $? ;;
  esac
done
