#!/bin/bash
# pipeline depth beyond 12 lanes (32 hardware queues): per-rank slices
export TMPDIR=/tmp
O=gpurun_out/${1:-r03n}
mkdir -p $O
for V in "" tools/var/libjxg_l24.so tools/var/libjxg_l30.so; do for H in 544 1088; do for M in host native; do
  env ${V:+JXG_LIB_PATH=$PWD/$V} JXG_BENCH_HW_QUEUES=32 JXG_SS_PROFILE=1 timeout -k 10 120 python -u tools/stream_probe.py --mode $M --world 1 --h $H --frames 300 --warmup 40 2>&1 | grep "mode\|rank" | sed "s|^|${V:-base} |" >> $O/probe.log || exit 1
done; done; done
