#!/bin/bash
# One GPU call: the GPU test suite, the headline bench, and the forced-bucket RCCL bench
# (DP diagnostics at one GPU).  Test failures (pytest rc 1) do not stop the call; a crash,
# fault or time limit (any other non-zero rc) ends it before anything else touches the GPU.
#   gpurun --timeout 1200 -- bash bench/gpu_session.sh <tag> [tests|bench|all]
TAG=${1:-cur}
WHAT=${2:-all}
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
if [ "$WHAT" = all ] || [ "$WHAT" = tests ]; then
  timeout -k 10 900 python3 -u -m pytest -v -m gpu --timeout 120 --timeout-method thread tests \
    > $O/tests.log 2>&1
  rc=$?
  tail -3 $O/tests.log
  if [ $rc -gt 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
fi
if [ "$WHAT" = all ] || [ "$WHAT" = bench ]; then
  timeout -k 10 300 python3 bench.py --steps 200 --warmup 20 > $O/bench.json 2> $O/bench.err \
    || { echo "bench failed"; tail -5 $O/bench.err; exit 1; }
  cat $O/bench.json
  timeout -k 10 300 python3 bench.py --steps 100 --warmup 10 --no-overhead --force-buckets \
    > $O/bench_fb.json 2> $O/bench_fb.err || { echo "forced-bucket bench failed"; tail -5 $O/bench_fb.err; exit 1; }
  cat $O/bench_fb.json
fi
