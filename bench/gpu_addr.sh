set -e
O=gpurun_out/addr; mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_native_gpu.py > $O/t.log 2>&1
rm -f $O/s.log
for S in "32 64 64 32 3 1 1" "32 512 512 4 3 1 1" "320 64 64 32 3 1 1" "320 512 512 4 3 1 1"; do
 MERCURY_EXT_PATH=mercury_amd/_C_stamps.so timeout -k 10 60 python3 bench/stamp_conv.py $S >> $O/s.log 2>&1
done
bash bench/ab_ext.sh mercury_amd/_C_old.so addr
