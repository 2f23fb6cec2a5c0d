#!/bin/bash
# Streams with and without super-frame batches (default build vs a variant
# whose batch-tile threshold admits larger frames), slices of the 8K frame
# and 1080p: ms/frame and the host time in submit / next_head / write_next.
# Usage: bash tools/batch_ab.sh TAG   (variant: tools/ab/libjxg_bt8k.so)
O=gpurun_out/$1; mkdir -p $O
for lib in "" tools/ab/libjxg_bt8k.so; do
  echo "== lib ${lib:-default}" >> $O/batch_ab.log
  for hh in 544 1088; do
    JXG_LIB_PATH=$lib timeout -k 10 150 python tools/stream_probe.py --mode host --world 1 --h $hh --frames 256 --warmup 48 >> $O/batch_ab.log 2>&1 || exit $?
  done
  JXG_LIB_PATH=$lib timeout -k 10 150 python tools/stream_probe.py --mode plain --w 1920 --h 1080 --frames 256 --warmup 64 >> $O/batch_ab.log 2>&1 || exit $?
done
