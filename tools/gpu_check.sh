#!/bin/bash
# GPU check on one box: GPU tests, smoke, default bench, rocprof kernel stats
# of the bench.  Usage: bash tools/gpu_check.sh TAG [extra bench args]
set -e
export TMPDIR=/tmp
R=$PWD
TAG=${1:-check}
shift || true
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 300 python bench.py "$@" > $O/bench.log 2>&1
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/$O/prof -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --alt-ans-streams 0 --alt-thesis 0 "$@" > $R/$O/bench_prof.log 2>&1
