set -e
mkdir -p gpurun_out/t1
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "prologue or conv_fwd" > gpurun_out/t1/k.log 2>&1
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_native_gpu.py > gpurun_out/t1/n.log 2>&1
mkdir -p gpurun_out/ab2
for i in 1 2; do
MERCURY_FUSE_BN_FWD=0 timeout -k 10 120 python3 bench.py --steps 300 --warmup 30 --no-overhead > gpurun_out/ab2/base$i.json 2>/dev/null
timeout -k 10 120 python3 bench.py --steps 300 --warmup 30 --no-overhead > gpurun_out/ab2/fused$i.json 2>/dev/null
done
