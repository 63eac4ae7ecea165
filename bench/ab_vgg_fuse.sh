# A/B: BN-apply folded into the next conv's prologue (fuse1) vs a separate bn_apply (fuse0), VGG11 speech, interleaved
set -e
O=gpurun_out/ab_vgg; mkdir -p $O
for i in 1 2 3; do
 for F in 0 1; do
  MERCURY_FUSE_BN_FWD=$F timeout -k 10 200 python3 bench.py --config vgg11-speech --steps 150 --warmup 15 --no-overhead > $O/f${F}_$i.json 2>/dev/null
 done
done
