# same-box A/B of env settings on the headline bench: bash bench/ab_env.sh TAG "ENV_A" "ENV_B" ...
set -e
T=$1; shift; O=gpurun_out/abenv_$T; mkdir -p $O
for i in 1 2; do
 j=0
 for E in "$@"; do
  j=$((j+1))
  env $E timeout -k 10 120 python3 bench.py --steps 300 --warmup 30 --no-overhead > $O/v${j}_$i.json 2>/dev/null
 done
done
