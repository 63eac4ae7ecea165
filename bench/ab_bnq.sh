# same-box A/B of a BN-kernel change: bn tests, bn_bench old/new, 3x headline bench old/new
#   bash bench/ab_bnq.sh OLD.so TAG
set -e
OLD=$1; O=gpurun_out/ab_$2; mkdir -p $O
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -m gpu -k "bn" > $O/t.log 2>&1
MERCURY_EXT_PATH=$OLD timeout -k 10 120 python3 bench/bn_bench.py > $O/bn_old.txt 2>&1
timeout -k 10 120 python3 bench/bn_bench.py > $O/bn_new.txt 2>&1
for i in 1 2 3; do
 MERCURY_EXT_PATH=$OLD timeout -k 10 120 python3 bench.py --steps 300 --warmup 30 --no-overhead > $O/old$i.json 2>/dev/null
 timeout -k 10 120 python3 bench.py --steps 300 --warmup 30 --no-overhead > $O/new$i.json 2>/dev/null
done
