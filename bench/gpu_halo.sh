set -e
O=gpurun_out/halo; mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "conv" > $O/t.log 2>&1
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_native_gpu.py > $O/n.log 2>&1
bash bench/ab_ext.sh mercury_amd/_C_old.so halo
