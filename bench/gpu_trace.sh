#!/bin/bash
# One GPU call: rocprofv3 kernel trace of the headline step -> per-kernel stats + per-queue
# timeline (marker: the once-per-step fused optimizer), then standalone graph replay times.
#   gpurun -- bash bench/gpu_trace.sh <tag> [extra bench.py args]
TAG=${1:-cur}; shift
OUT=gpurun_out/trace_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- \
  python3 bench.py --steps 60 --warmup 10 --no-overhead "$@" > $OUT/bench.log 2>&1 || exit 1
python3 bench/trace_timeline.py $OUT/trace optimizer_fused 40 > $OUT/timeline.txt || exit 1
cat $OUT/timeline.txt | head -40
timeout -k 10 240 python3 bench/host_overhead.py > $OUT/host_overhead.log 2>&1 || exit 1
cat $OUT/host_overhead.log | tail -12
