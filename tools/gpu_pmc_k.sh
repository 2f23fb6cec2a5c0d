#!/bin/bash
# PMC passes (one counter group per pass) for one kernel regex.
# Usage: bash tools/gpu_pmc_k.sh OUTDIR REGEX [bench args...]
set -e
OUT=$1; K=$2; shift 2
EXTRA=("$@")
mkdir -p $OUT
export TMPDIR=/tmp
R=$PWD
run() { timeout -k 10 120 rocprofv3 --pmc $2 --kernel-include-regex "$K" -d $R/$OUT/$1 -o run --output-format csv -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline "${EXTRA[@]}" > $R/$OUT/$1.log 2>&1; }
run p1 "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY"
run p4 "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE SQ_INSTS_VMEM SQ_INSTS_BRANCH"
