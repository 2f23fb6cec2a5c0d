#!/bin/bash
# Round 3: debug the 2-rank ShardStream run, then parity of the kernel
# changes, the GPU suite, the default bench and the gloo 2-rank bench.
set -e
export TMPDIR=/tmp
O=gpurun_out/${1:-r03c}
mkdir -p $O
timeout -k 10 150 python -u tools/dbg_stream2.py stream > $O/dbg_stream.log 2>&1
timeout -k 10 150 python -u tools/dbg_stream2.py sync > $O/dbg_sync.log 2>&1
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -x -v --timeout 200 --timeout-method thread > $O/parity.log 2>&1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread --deselect tests/test_gpu_parity.py --deselect tests/test_gpu_configs.py > $O/gpu_tests.log 2>&1
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 > $O/bench.log 2>&1
JXG_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 20 --warmup 2 > $O/bench_gloo2.log 2>&1
