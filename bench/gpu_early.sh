set -e
O=gpurun_out/early; mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_native_gpu.py tests/test_native_dp_gpu.py tests/test_rccl_gpu.py > $O/t.log 2>&1
bash bench/ab_env.sh early "MERCURY_EARLY_OPT=0" "MERCURY_EARLY_OPT=1"
