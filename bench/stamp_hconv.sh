for v in variants/st_base.so variants/st_baseDHC_NO_TRANSFORM.so variants/st_baseDHC_NO_COEF.so; do
  echo "== $v"
  for args in "320 64 64 32 1 128 64 1 0" "320 64 64 32 1 128 64 1 1"; do
    MERCURY_EXT_PATH=$PWD/$v timeout -k 10 120 python3 bench/stamp_hconv.py $args | grep -E "shape|mainloop|loop split" || exit 1
  done
done
