#!/bin/bash
# Round 3: parity of the product (X / B packed candidate passes), then the
# kernel A/B, the GPU suite, the default bench, the gloo 2-rank streamed-shard
# bench and the 2-process streamed-frames test.
set -e
export TMPDIR=/tmp
O=gpurun_out/${1:-r03g}; shift
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -x -v --timeout 200 --timeout-method thread > $O/parity.log 2>&1
for L in "" "$@"; do
  n=${L:-product}; n=$(basename $n .so)
  env ${L:+JXG_LIB_PATH=$PWD/$L} timeout -k 10 120 python -u bench.py --no-pipeline --steps 10 --warmup 2 --no-cpu-baseline --no-quality --alt-thesis 0 --alt-coder 0 > $O/iso_$n.log 2>&1
  env ${L:+JXG_LIB_PATH=$PWD/$L} timeout -k 10 150 python -u bench.py --steps 60 --warmup 3 --no-cpu-baseline --no-quality --alt-thesis 0 --alt-coder 0 > $O/pipe_$n.log 2>&1
done
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread --deselect tests/test_gpu_shard.py::test_multiprocess_streamed_frames > $O/gpu_tests.log 2>&1
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 > $O/bench.log 2>&1
JXG_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 20 --warmup 2 > $O/bench_gloo2.log 2>&1
timeout -k 10 200 python -u -m pytest tests/test_gpu_shard.py::test_multiprocess_streamed_frames -x -v -s --timeout 170 --timeout-method thread > $O/mp_stream_test.log 2>&1
