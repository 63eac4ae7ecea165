#!/bin/bash
# Generic GPU call: run the given pytest targets (if any), then each extra python script,
# every step under its own time limit; a crash / fault / time limit ends the call.
#   gpurun -- bash bench/gpu_run.sh <tag> "<pytest targets or ->" "<script 1 args>" ...
TAG=$1; shift
T=$1; shift
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
if [ "$T" != "-" ]; then
  timeout -k 10 600 python3 -u -m pytest -v -m gpu --timeout 120 --timeout-method thread $T \
    > $O/tests.log 2>&1
  rc=$?
  grep -E "PASSED|FAILED|ERROR|passed|failed" $O/tests.log | tail -40
  if [ $rc -gt 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
fi
i=0
for S in "$@"; do
  i=$((i+1))
  timeout -k 10 400 python3 -u $S > $O/run$i.out 2> $O/run$i.err
  rc=$?
  cat $O/run$i.out | tail -40
  if [ $rc -ne 0 ]; then echo "step $i ($S) rc=$rc"; tail -20 $O/run$i.err; exit $rc; fi
done
