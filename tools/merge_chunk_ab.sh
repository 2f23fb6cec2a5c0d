#!/bin/bash
# merge_eval's per-XCD tile chunk (JXG_MERGE_CHUNK): merge-stage time and
# the XYB re-fetch (PMC FETCH_SIZE) per chunk size, variants interleaved.
# Build here: bash tools/merge_chunk_ab.sh build ; on the box: bash tools/merge_chunk_ab.sh run TAG
set -e
D=$(cd "$(dirname "$0")/.." && pwd)
if [ "$1" = build ]; then
  for c in 8 16 32 64; do
    bash $D/tools/build_variant.sh chunk$c "-DJXG_MERGE_CHUNK=$c"
    mkdir -p $D/tools/ab && mv $D/tools/var/libjxg_chunk$c.so $D/tools/ab/
  done
  exit 0
fi
O=$D/gpurun_out/$2/merge_chunk
mkdir -p $O
export TMPDIR=/tmp
for round in 1 2; do
  for c in 8 16 32 64; do
    echo "== chunk $c round $round" >> $O/probe.log
    JXG_LIB_PATH=$D/tools/ab/libjxg_chunk$c.so timeout -k 10 120 python tools/merge_probe.py >> $O/probe.log 2>&1
  done
done
for c in 16 32 64; do
  JXG_LIB_PATH=$D/tools/ab/libjxg_chunk$c.so timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_$c -o run -- python3 tools/merge_probe.py > $O/pmc_$c.log 2>&1
done
