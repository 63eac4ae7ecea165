# round-end check: every gpu test, smoke(), default bench, and a kernel-trace profile
set -e
O=gpurun_out/final; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread tests > $O/tests.log 2>&1
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 300 python3 bench.py > $O/bench.json 2>$O/bench.err
bash bench/gpu_profile.sh r1e > $O/profile.log 2>&1
