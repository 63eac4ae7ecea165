set -o pipefail
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/s26; mkdir -p $O
T="--timeout 120 --timeout-method thread"
timeout -k 10 600 python3 -u -m pytest tests -m gpu -q $T > $O/tests.txt 2>&1; rc=$?; tail -n 3 $O/tests.txt; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -n 20 $O/smoke.log; exit 1; }
timeout -k 10 300 python3 bench.py --steps 300 --warmup 30 > $O/bench_r18.json 2>&1 || exit 1
tail -n 1 $O/bench_r18.json
timeout -k 10 120 python3 -u bench/queue_probe.py > $O/queue_probe.txt 2>&1 || exit 1
timeout -k 10 300 python3 bench.py --steps 300 --warmup 30 --force-buckets --no-overhead > $O/bench_r18_dp.json 2>&1 || exit 1
for c in mobilenetv2-cifar100 vgg11-speech resnet50-imagenet; do
timeout -k 10 400 python3 bench.py --config $c --steps 100 --warmup 10 > $O/$c.json 2>&1 || exit 1
done
for m in train score; do
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tr_mbv2_$m -- python3 bench.py --config mobilenetv2-cifar100 --replay-only $m --steps 30 --warmup 5 > $O/tr_mbv2_$m.log 2>&1 || exit 1
mk=step_begin_kernel; [ $m = score ] && mk=pool_build_kernel; python3 bench/seq_trace.py $O/tr_mbv2_$m $mk 20 > $O/seq_mbv2_$m.txt 2>&1 || true
done
echo done
