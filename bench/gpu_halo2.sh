set -e
O=gpurun_out/halo2; mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py > $O/t.log 2>&1
for i in 1 2; do timeout -k 10 120 python3 bench.py --steps 300 --warmup 30 --no-overhead > $O/b$i.json 2>/dev/null; done
