set -e
O=gpurun_out/presets; mkdir -p $O
for C in mobilenetv2-cifar100 resnet50-imagenet vgg11-speech; do
 for F in 0 1; do
  MERCURY_FUSE_BN_FWD=$F timeout -k 10 300 python3 bench.py --config $C --steps 100 --warmup 10 --no-overhead > $O/${C}_fuse$F.json 2>$O/${C}_fuse$F.err
 done
done
timeout -k 10 300 python3 bench.py --steps 300 --warmup 30 > $O/resnet18.json 2>/dev/null
