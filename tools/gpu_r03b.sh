#!/bin/bash
# Round 3: kernel A/B (front: CfL DCT8 reuse + packed quantization; merge:
# two-plane LDS, 4 workgroups / CU) -- bit-exact parity of the product first,
# then one-at-a-time (kernel times) and pipelined benches of each library.
set -e
export TMPDIR=/tmp
O=gpurun_out/${1:-r03b}; shift
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -x -q --timeout 200 --timeout-method thread > $O/parity.log 2>&1
for L in "" "$@"; do
  n=${L:-product}; n=$(basename $n .so)
  env ${L:+JXG_LIB_PATH=$PWD/$L} timeout -k 10 120 python -u bench.py --no-pipeline --steps 10 --warmup 2 --no-cpu-baseline --no-quality --alt-thesis 0 --alt-coder 0 > $O/iso_$n.log 2>&1
done
for L in "" "$@"; do
  n=${L:-product}; n=$(basename $n .so)
  env ${L:+JXG_LIB_PATH=$PWD/$L} timeout -k 10 150 python -u bench.py --steps 60 --warmup 3 --no-cpu-baseline --no-quality --alt-thesis 0 --alt-coder 0 > $O/pipe_$n.log 2>&1
done
