#!/bin/bash
# Front-kernel timing experiments: the product library against variant builds
# (tools/ab/libjxg_NAME.so), front kernel ms per launch at effort 7 and 4.
# Usage: bash tools/load_ab.sh TAG NAME...
set -e
O=gpurun_out/$1; shift
mkdir -p $O
for r in 1 2; do
  for n in base "$@"; do
    L=$PWD/jpeg-xl-lossy-image-compression-thesis_amd/jxg/libjxg.so
    [ $n != base ] && L=$PWD/tools/ab/libjxg_$n.so
    for e in 7 4; do
      echo "== $n e$e" >> $O/ab.log
      PROBE_MERGE=1 JXG_LIB_PATH=$L timeout -k 10 120 python tools/front_phase_probe.py $e cjxl 8 >> $O/ab.log 2>&1
    done
  done
done
