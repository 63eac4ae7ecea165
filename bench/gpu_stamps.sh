set -e
O=gpurun_out/stamps; mkdir -p $O
for S in "32 64 64 32 3 1 1" "32 128 128 16 3 1 1" "32 512 512 4 3 1 1" "32 64 128 32 1 2 0" "320 64 64 32 3 1 1" "320 128 128 16 3 1 1" "320 512 512 4 3 1 1"; do
 MERCURY_EXT_PATH=mercury_amd/_C_stamps.so timeout -k 10 60 python3 bench/stamp_conv.py $S >> $O/s.log 2>&1
done
