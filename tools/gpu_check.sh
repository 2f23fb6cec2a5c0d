#!/bin/bash
# One GPU-box pass: GPU tests, smoke, the default bench (CPU baseline with a
# thread sweep), and a 4-rank gloo rehearsal of bench.py's default sharded
# path on the box's one GPU (bench.py starts the ranks itself).
# Usage: bash tools/gpu_check.sh TAG [tests|tcjxl|bench|bench20|gloo|rank8|chainab|cfg|small ...]
# (default: tests bench gloo)
set -e
export TMPDIR=/tmp
TAG=${1:-check}; shift || true
STEPS=${@:-tests bench gloo}
O=gpurun_out/$TAG
mkdir -p $O
for s in $STEPS; do
  case $s in
    tests) timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1
           timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 ;;
    tcjxl) timeout -k 10 400 python -u -m pytest tests/test_gpu_cli.py tests/test_gpu_configs.py -m gpu -x -v -k "cjxl or cli or c_abi" --timeout 200 --timeout-method thread > $O/gpu_tests_cjxl.log 2>&1 ;;
    bench) timeout -k 10 300 python bench.py --cpu-sweep 16,32,64,128,256 > $O/bench.log 2>&1 ;;
    bench20) timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-quality > $O/bench20.log 2>&1 ;;
    gloo) JXG_DIST_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 4 --steps 20 --warmup 3 > $O/bench_gloo4.log 2>&1 ;;
    rank8) # rank 7's real kind-1 shard of an 8K frame over 8 ranks, one context
           for pr in cjxl plain; do
             timeout -k 10 150 python tools/stream_probe.py --mode rank --world 8 --preset $pr --frames 200 --warmup 32 >> $O/probe_rank8.log 2>&1
           done ;;
    chainab) # same-box A/B of tools/ab builds (tools/build_lib_variant.sh): stage times
           for r in 1 2; do for v in $AB; do
             JXG_LIB_PATH=$PWD/tools/ab/libjxg_$v.so timeout -k 10 120 python tools/chain_probe.py >> $O/chain_ab.log 2>&1
           done; done ;;
    rankprof) # API + kernel + copy trace of rank 7's shard stream and of the 7680x544 slice
           timeout -k 10 200 rocprofv3 --hip-trace --kernel-trace --memory-copy-trace --stats --output-format csv -d $O/prof_rank7 -o run -- python3 tools/stream_probe.py --mode rank --world 8 --preset plain --frames 100 --warmup 16 > $O/prof_rank7.log 2>&1
           timeout -k 10 200 rocprofv3 --hip-trace --kernel-trace --memory-copy-trace --stats --output-format csv -d $O/prof_slice -o run -- python3 tools/stream_probe.py --mode host --world 1 --h 544 --preset plain --frames 100 --warmup 16 > $O/prof_slice.log 2>&1 ;;
    cfg) bash tools/gpu_configs.sh $TAG/cfg ;;
    small) # small-frame streams: config 3's 1080p frames, a 1/8 slice of the
           # 8K frame (one rank's load), the 8-context emulation; then a
           # kernel + copy trace of the 1080p stream
           timeout -k 10 150 python tools/stream_probe.py --mode plain --w 1920 --h 1080 --frames 256 --warmup 32 > $O/probe_1080p.log 2>&1
           for hh in 544 1088 2160 4320; do
             timeout -k 10 150 python tools/stream_probe.py --mode host --world 1 --h $hh --frames 256 --warmup 32 >> $O/probe_slices.log 2>&1
           done
           timeout -k 10 150 python tools/stream_probe.py --mode host --world 8 --frames 40 > $O/probe_ctx8.log 2>&1
           timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --hip-trace --stats --output-format csv -d $O/prof_1080p -o run -- python3 tools/stream_probe.py --mode plain --w 1920 --h 1080 --frames 64 --warmup 8 > $O/prof_1080p.log 2>&1 ;;
  esac
done
