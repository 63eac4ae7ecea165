# re-entry check after a container rebuild: every gpu test, smoke(), the default bench,
# and a kernel-trace profile of the headline step
set -e
O=gpurun_out/reentry; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread tests > $O/tests.log 2>&1
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 300 python3 bench.py > $O/bench.json 2>$O/bench.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- \
  python3 bench.py --steps 60 --warmup 10 --no-overhead > $O/prof_bench.log 2>&1
python3 bench/trace_timeline.py $O/trace optimizer_kernel 40 > $O/timeline.txt
