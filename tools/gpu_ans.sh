#!/bin/bash
# ANS coder iteration: ANS parity tests, the ANS bench line, kernel stats
set -e
export TMPDIR=/tmp
R=$PWD
O=gpurun_out/${1:-ans}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "ans or config" > $O/tests.log 2>&1
timeout -k 10 300 python bench.py --no-cpu-baseline --no-quality --coder ans --alt-ans-streams 0 --alt-thesis 0 > $O/bench_ans.log 2>&1
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/$O/prof -o run --output-format csv -- python3 $R/bench.py --steps 6 --warmup 2 --no-cpu-baseline --no-quality --coder ans --alt-ans-streams 0 --alt-thesis 0 > $R/$O/bench_prof.log 2>&1
