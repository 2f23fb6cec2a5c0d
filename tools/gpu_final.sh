#!/bin/bash
# Round evidence on one GPU box: GPU tests, smoke, default bench (with the CPU
# baseline), rocprofv3 kernel stats of the same bench, PMC HBM-traffic passes
# of the front kernel.  Usage: bash tools/gpu_final.sh TAG
set -e
export TMPDIR=/tmp
TAG=${1:-final}
R=$PWD
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 300 python bench.py > $O/bench.log 2>&1
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/$O/prof -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --alt-ans-streams 0 --alt-thesis 0 > $R/$O/bench_prof.log 2>&1
cd /tmp && timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex front_kernel -d $R/$O/pmc_fetch -o run --output-format csv -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --alt-ans-streams 0 --alt-thesis 0 > $R/$O/pmc_fetch.log 2>&1
cd /tmp && timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex front_kernel -d $R/$O/pmc_write -o run --output-format csv -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --alt-ans-streams 0 --alt-thesis 0 > $R/$O/pmc_write.log 2>&1
