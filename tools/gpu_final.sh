#!/bin/bash
# Round evidence on one GPU box: GPU tests, smoke, default bench (with the CPU
# baseline and the decoded-quality check), rocprofv3 kernel stats of the same
# bench, PMC passes (front kernel: instructions, waits, HBM traffic; merge_eval:
# instructions), the BASELINE configs at N = 1 and a 2-rank gloo rehearsal of
# the multi-GPU bench.  Usage: bash tools/gpu_final.sh TAG
set -e
export TMPDIR=/tmp
TAG=${1:-final}
PART=${2:-all}  # a: tests, smoke, bench, trace, gloo2; b: PMC passes, configs
R=$PWD
O=gpurun_out/$TAG
mkdir -p $O
if [ "$PART" != b ]; then
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 300 python bench.py > $O/bench.log 2>&1
cd /tmp && GPU_MAX_HW_QUEUES=16 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/$O/prof -o run --output-format csv -- python3 $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-quality --no-single --alt-coder 0 --alt-thesis 0 > $R/$O/bench_prof.log 2>&1
cd $R
JXG_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 2 --no-cpu-baseline > $O/bench_gloo2.log 2>&1
fi
if [ "$PART" != a ]; then
KERNEL=front_kernel bash profiles/pmc_front.sh $O/pmc_front
BENCH_ARGS="--steps 2 --warmup 1 --no-cpu-baseline --no-quality --no-single --alt-coder 0 --alt-thesis 0 --alt-cjxl 0 --alt-e4 0 --no-pipeline" \
  KERNEL=merge_eval_kernel bash profiles/pmc_front.sh $O/pmc_eval
bash tools/gpu_configs.sh $TAG/cfg
fi
