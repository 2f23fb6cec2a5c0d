#!/bin/bash
# Sanitizer run of the CPU suite: the host code of
# the product (bit writers, TOC, payload heads, shard plan / assembly: libjxg.so
# built with host-side ASan + UBSan) and the oracle (ASan + UBSan), each under
# its own runtime preloaded into python (gcc's for the oracle, clang's for
# libjxg -- one ASan runtime per process).  Usage: bash tools/asan_suite.sh OUTDIR
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
O=${1:-$R/profiles/r03_asan}
mkdir -p $O
make -s -C $R/jpeg-xl-lossy-image-compression-thesis_amd asan
make -s -C $R/oracle asan
export ASAN_OPTIONS=detect_leaks=0:abort_on_error=1:halt_on_error=1
export UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1
cd $R
# 1. oracle restatement (+ the native prefix-parity test binary) under gcc's runtime
JXO_LIB_PATH=$R/oracle/asan/liboracle.so \
JXG_NATIVE_CFLAGS="-fsanitize=address,undefined -fno-sanitize-recover=undefined -fno-omit-frame-pointer" \
LD_PRELOAD="$(gcc -print-file-name=libasan.so) $(gcc -print-file-name=libubsan.so)" \
  python -m pytest tests -m "not gpu" -q -p no:cacheprovider \
    --deselect tests/test_shard_host.py --deselect tests/test_abi_harness.py \
    > $O/oracle_asan.log 2>&1 && echo "oracle: ok" || { echo "oracle: FAILED"; tail -30 $O/oracle_asan.log; exit 1; }
# 2. libjxg host code under clang's runtime (shard plan, payload heads, host
#    assembly incl. malformed version-2 heads, the ABI exports)
CLANG_ASAN=$(ls /opt/rocm/lib/llvm/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so | head -1)
JXG_LIB_PATH=$R/jpeg-xl-lossy-image-compression-thesis_amd/build-asan/libjxg.so \
LD_PRELOAD="$CLANG_ASAN" \
  python -m pytest tests/test_shard_host.py tests/test_abi_harness.py -m "not gpu" -q -p no:cacheprovider \
    > $O/libjxg_asan.log 2>&1 && echo "libjxg host: ok" || { echo "libjxg host: FAILED"; tail -30 $O/libjxg_asan.log; exit 1; }
tail -n 2 $O/oracle_asan.log $O/libjxg_asan.log
