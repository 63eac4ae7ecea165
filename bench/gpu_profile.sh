#!/bin/bash
# One GPU call: kernel trace of the headline step + per-queue timeline, standalone graph
# replays, and graph-timed per-layer plan sweeps at the train and scoring batch.
#   gpurun -- bash bench/gpu_profile.sh [tag]
set -e
TAG=${1:-cur}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- \
  python3 bench.py --steps 60 --warmup 10 --no-overhead > $OUT/bench.log 2>&1
python3 bench/trace_timeline.py $OUT/trace optimizer_kernel 40 > $OUT/timeline.txt
timeout -k 10 240 python3 bench/host_overhead.py > $OUT/host_overhead.log 2>&1
timeout -k 10 400 python3 bench/kernel_sweep.py --batch 32 --write-cache $OUT/tune32.json \
  > $OUT/sweep32.jsonl 2>&1
timeout -k 10 400 python3 bench/kernel_sweep.py --batch 320 --kind fwd --write-cache $OUT/tune320.json \
  > $OUT/sweep320.jsonl 2>&1
