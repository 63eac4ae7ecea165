# one PMC pass (8 SQ counters) over the headline ResNet-18 IS step: MFMA busy vs wave cycles per kernel
set -e
O=gpurun_out/pmc_step; mkdir -p $O
export TMPDIR=/tmp
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_ANY --output-format csv -d $O/p1 -o run -- python3 bench.py --steps 10 --warmup 3 --no-overhead > $O/p1.log 2>&1
