#!/bin/bash
# Same-box A/B of library builds on the default 8K stream (60 timed frames,
# no side lines), interleaved: bash tools/bench_ab.sh TAG lib1 lib2 ...
# ("" = the product build)
O=gpurun_out/$1; shift; mkdir -p $O
for r in 1 2; do
  for lib in "$@"; do
    echo "== ${lib:-default} round $r" >> $O/bench_ab.log
    JXG_LIB_PATH=$lib timeout -k 10 200 python bench.py --steps 60 --warmup 5 --no-cpu-baseline --no-quality --alt-coder 0 --alt-thesis 0 --alt-cjxl 0 > $O/tmp.log 2>&1 || exit $?
    grep -o '"value": [0-9.]*\|"ms_latency": [0-9.]*' $O/tmp.log | head -2 | tr '\n' ' ' >> $O/bench_ab.log; echo >> $O/bench_ab.log
  done
done
