#!/bin/bash
# Submit one gpurun call; when the pool reports no free box (status=transient:
# nothing ran, nothing charged) wait and submit the same call again, up to 8
# times.  A call that ran (any other status) is never repeated.
# Usage: tools/gpurun_q.sh OUTFILE TIMEOUT 'command'
OUT=$1; TO=$2; CMD=$3
for i in 1 2 3 4 5 6 7 8; do
  /usr/local/graft/bin/gpurun --timeout $TO -- "$CMD" > $OUT 2>&1
  if grep -q "status=transient" $OUT; then sleep 150; continue; fi
  break
done
echo done >> $OUT
