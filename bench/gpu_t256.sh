set -e
O=gpurun_out/t256; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -m gpu -k "all_tiles or pipelined" > $O/tests.log 2>&1
timeout -k 10 400 python3 bench/kernel_sweep.py --batch 320 --kind fwd --pipes 0 > $O/sweep320.jsonl 2>&1
