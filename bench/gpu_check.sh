set -e
O=gpurun_out/chk; mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_native_gpu.py > $O/t.log 2>&1
for i in 1 2; do timeout -k 10 120 python3 bench.py --steps 300 --warmup 30 --no-overhead > $O/b$i.json 2>/dev/null; done
timeout -k 10 400 python3 bench/kernel_sweep.py --batch 32 --pipes 0 > $O/sweep32.jsonl 2>&1
timeout -k 10 400 python3 bench/kernel_sweep.py --batch 320 --kind fwd --pipes 0 > $O/sweep320.jsonl 2>&1
