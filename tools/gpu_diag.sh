#!/bin/bash
# Parity diagnosis on the box: section-level GPU vs oracle comparison, then the
# parity suites file by file (a test failure continues; a timeout, abort or
# signal stops the script).  Usage: bash tools/gpu_diag.sh TAG [test files...]
export TMPDIR=/tmp
O=gpurun_out/$1; shift
mkdir -p $O
timeout -k 10 150 python tools/diag_sections.py > $O/diag.log 2>&1
rc=$?; echo "diag rc=$rc" >> $O/diag.log
[ $rc -ge 124 ] && exit $rc
for t in "$@"; do
  timeout -k 10 300 python -u -m pytest $t -x -q --timeout 120 --timeout-method thread > $O/$(basename $t .py).log 2>&1
  rc=$?; echo "$t rc=$rc" >> $O/summary.log
  [ $rc -ge 124 ] && exit $rc
done
exit 0
