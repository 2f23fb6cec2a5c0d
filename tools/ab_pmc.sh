#!/bin/bash
# PMC A/B of experiment builds for one kernel: bash tools/ab_pmc.sh TAG REGEX name1 name2 ...
set -e
export TMPDIR=/tmp
TAG=$1; K=$2; shift 2
R=$PWD
mkdir -p gpurun_out/$TAG
for n in "$@"; do
  if [ "$n" = prod ]; then L=$R/jpeg-xl-lossy-image-compression-thesis_amd/jxg/libjxg.so; else L=$R/tools/exp/libjxg_$n.so; fi
  i=0
  for ctr in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY" \
             "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE SQ_INSTS_VMEM SQ_INSTS_BRANCH"; do
    i=$((i+1))
    cd /tmp && JXG_LIB_PATH=$L timeout -k 10 120 rocprofv3 --pmc $ctr --kernel-include-regex "$K" -d $R/gpurun_out/$TAG/${n}_p$i -o run --output-format csv -- python3 $R/tools/mprof_run.py 2 > $R/gpurun_out/$TAG/${n}_p$i.log 2>&1
    cd $R
  done
done
