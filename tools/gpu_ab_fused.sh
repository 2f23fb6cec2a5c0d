#!/bin/bash
# parity of a library build (GPU tests with JXG_LIB_PATH) + kernel stats A/B
set -e
export TMPDIR=/tmp
TAG=$1; NEW=$2; OLD=$3
mkdir -p gpurun_out/$TAG
JXG_LIB_PATH=$PWD/$NEW timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -x -q --timeout 200 --timeout-method thread > gpurun_out/$TAG/parity.log 2>&1
bash tools/gpu_ab_kstats.sh $TAG $OLD $NEW
