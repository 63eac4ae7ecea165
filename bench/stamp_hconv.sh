export MERCURY_EXT_PATH=$PWD/variants/stamps.so
for args in "320 64 64 32 1" "320 256 256 8 1 256 128 1"; do
  timeout -k 10 120 python3 bench/stamp_hconv.py $args || exit 1
done
timeout -k 10 120 python3 bench/stamp_conv.py 320 64 64 32 3 1 1 || exit 1
