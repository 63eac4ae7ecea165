# in-situ step tuning, then A/B of bench.py with and without the tuned cache
set -e
O=gpurun_out/stune; mkdir -p $O
timeout -k 10 780 python3 -u bench/step_tune.py --out $O/cache.json --budget ${BUDGET:-540} > $O/tune.log 2>&1
for i in 1 2 3; do
 timeout -k 10 120 python3 bench.py --steps 300 --warmup 30 --no-overhead > $O/base$i.json 2>/dev/null
 MERCURY_TUNE_CACHE=$O/cache.json timeout -k 10 120 python3 bench.py --steps 300 --warmup 30 --no-overhead > $O/tuned$i.json 2>/dev/null
done
