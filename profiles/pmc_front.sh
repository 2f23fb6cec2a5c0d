#!/bin/bash
# PMC passes over the front kernel (one counter group per pass; no trace
# domains mixed with --pmc).  Usage: bash profiles/pmc_front.sh OUTDIR
set -e
OUT=${1:-gpurun_out/pmc}
mkdir -p $OUT
export TMPDIR=/tmp
R=$PWD
# one-at-a-time encodes (each kernel alone on the GPU), no side measurements
BARGS=${BENCH_ARGS:---steps 2 --warmup 1 --no-cpu-baseline --no-quality --alt-coder 0 --alt-thesis 0 --alt-cjxl 0 --no-pipeline}
run() { timeout -k 10 300 rocprofv3 --pmc $2 --kernel-include-regex "$3" -d $R/$OUT/$1 -o run --output-format csv -- python3 $R/bench.py $BARGS > $R/$OUT/$1.log 2>&1; }
K=${KERNEL:-front_kernel}
run p1 "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY" "$K"
run p2 "FETCH_SIZE" "$K"
run p3 "WRITE_SIZE" "$K"
run p4 "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE" "$K"
