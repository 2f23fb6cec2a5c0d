#!/bin/bash
export TMPDIR=/tmp
O=gpurun_out/${1:-r03y}
mkdir -p $O
JXG_LIB_PATH=$PWD/tools/var/libjxg_pprof.so timeout -k 10 300 python -u bench.py --config 3 --steps 4 --warmup 1 --no-cpu-baseline --no-quality --alt-thesis 0 --alt-coder 0 > $O/cfg3_pprof.log 2>&1
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $GRAFT_REPO_ROOT/$O/prof3 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --config 3 --steps 2 --warmup 1 --no-cpu-baseline --no-quality --alt-thesis 0 --alt-coder 0 > $GRAFT_REPO_ROOT/$O/prof3.log 2>&1
