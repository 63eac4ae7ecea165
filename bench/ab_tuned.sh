set -e
mkdir -p gpurun_out/ab1
for i in 1 2; do
timeout -k 10 120 python3 bench.py --steps 300 --warmup 30 --no-overhead > gpurun_out/ab1/base$i.json 2>/dev/null
MERCURY_TUNE_CACHE=bench/tuned_cache_r1c.json MERCURY_TUNE_SAVE=0 timeout -k 10 120 python3 bench.py --steps 300 --warmup 30 --no-overhead > gpurun_out/ab1/tuned$i.json 2>/dev/null
done
