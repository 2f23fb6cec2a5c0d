#!/bin/bash
# PMC passes over the front kernel (one counter group per pass; no trace
# domains mixed with --pmc).  Usage: bash profiles/pmc_front.sh OUTDIR
set -e
OUT=${1:-gpurun_out/pmc}
mkdir -p $OUT
export TMPDIR=/tmp
R=$PWD
# one-at-a-time encodes (each kernel alone on the GPU), no side measurements
BARGS=${BENCH_ARGS:---steps 2 --warmup 1 --no-cpu-baseline --no-quality --no-single --alt-coder 0 --alt-thesis 0 --alt-cjxl 0 --alt-e4 0 --no-pipeline}
run() { timeout -k 10 300 rocprofv3 --pmc $2 --kernel-include-regex "$3" -d $R/$OUT/$1 -o run --output-format csv -- python3 $R/bench.py $BARGS > $R/$OUT/$1.log 2>&1; }
K=${KERNEL:-front_kernel}
run p1 "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY" "$K"
run p2 "FETCH_SIZE" "$K"
run p3 "WRITE_SIZE" "$K"
run p4 "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE" "$K"
# EXTRA=1: stall attribution (memory-instruction levels = outstanding
# instructions per cycle, so LEVEL / INSTS = mean latency in cycles;
# instruction fetch; L2 hit rate; L1 -> L2 read latency)
if [ -n "$EXTRA" ]; then
  run p5 "SQ_INSTS_VMEM_RD SQ_INST_LEVEL_VMEM SQ_INST_LEVEL_LDS SQ_IFETCH SQ_IFETCH_LEVEL SQ_INSTS_SMEM SQ_INST_LEVEL_SMEM SQ_ACTIVE_INST_ANY" "$K"
  run p6 "SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM_RD SQ_LDS_DATA_FIFO_FULL SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_INSTS_BRANCH" "$K"
  run p7 "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_DRAM_sum TCC_READ_sum" "$K"
  run p8 "TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_PENDING_STALL_CYCLES_sum" "$K"
fi
