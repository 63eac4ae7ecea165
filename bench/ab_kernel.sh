# same-box A/B of two extension builds on a microbenchmark: bash bench/ab_kernel.sh OLD.so TAG CMD...
set -e
old=$1; tag=$2; shift 2; o=gpurun_out/abk_${tag}; mkdir -p $o
for r in 1 2 3; do
  MERCURY_EXT_PATH=$old timeout -k 10 200 "$@" > $o/old$r.json 2> $o/old$r.err
  timeout -k 10 200 "$@" > $o/new$r.json 2> $o/new$r.err
done
tail -n 1 $o/old*.json $o/new*.json
