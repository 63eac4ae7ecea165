set -e
O=gpurun_out/tchk; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread tests/test_native_gpu.py tests/test_kernels_gpu.py > $O/t.log 2>&1
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_ANY --output-format csv -d $O/p1 -o run -- python3 bench.py --steps 10 --warmup 3 --no-overhead > $O/p1.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 bench.py --steps 60 --warmup 10 --no-overhead > $O/prof_bench.log 2>&1
for i in 1 2; do timeout -k 10 200 python3 bench.py --steps 300 --warmup 30 --no-overhead > $O/b$i.json 2>/dev/null; done
