# same-box A/B of two builds on the headline bench only: bash bench/ab_quick.sh OLD.so TAG
set -e
OLD=$1; O=gpurun_out/ab_$2; mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_native_gpu.py > $O/t.log 2>&1
for i in 1 2 3; do
 MERCURY_EXT_PATH=$OLD timeout -k 10 120 python3 bench.py --steps 300 --warmup 30 --no-overhead > $O/old$i.json 2>/dev/null
 timeout -k 10 120 python3 bench.py --steps 300 --warmup 30 --no-overhead > $O/new$i.json 2>/dev/null
done
