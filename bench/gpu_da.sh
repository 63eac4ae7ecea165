# direct-A (pipe 1) conv loop: numerics, then per-shape fwd times vs the register-staged loop
set -e
O=gpurun_out/da; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -m gpu -k "pipelined or conv_fwd or conv_bwd" > $O/tests.log 2>&1
timeout -k 10 300 python3 bench/kernel_sweep.py --batch 320 --kind fwd --pipes 0,1 > $O/sweep320.jsonl 2>&1
timeout -k 10 300 python3 bench/kernel_sweep.py --batch 32 --kind fwd --pipes 0,1 > $O/sweep32.jsonl 2>&1
