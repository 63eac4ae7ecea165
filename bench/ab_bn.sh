set -e
O=gpurun_out/ab_bn; mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "bn or native" tests/test_native_gpu.py > $O/t.log 2>&1
MERCURY_EXT_PATH=mercury_amd/_C_old.so timeout -k 10 200 python3 bench/bn_bench.py > $O/old_bn.log 2>&1
timeout -k 10 200 python3 bench/bn_bench.py > $O/new_bn.log 2>&1
bash bench/ab_quick.sh mercury_amd/_C_old.so bnq
