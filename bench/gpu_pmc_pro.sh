set -e
export TMPDIR=/tmp
O=gpurun_out/pmc3; mkdir -p $O
timeout -k 10 200 python3 bench/pro_bench.py > $O/pro.log 2>&1
timeout -k 10 200 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k prologue > $O/t.log 2>&1
for S in "320 64 64 32 3 1 1 20" "32 64 64 32 3 1 1 20"; do
 T=$(echo $S | tr ' ' _)
 timeout -s KILL 60 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_BUSY_CYCLES --output-format csv -d $O/p1_$T -o run -- python3 bench/conv_once.py $S > $O/p1_$T.log 2>&1
 timeout -s KILL 60 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE --output-format csv -d $O/p2_$T -o run -- python3 bench/conv_once.py $S > $O/p2_$T.log 2>&1
 timeout -s KILL 60 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCP_TOTAL_CACHE_ACCESSES_sum TA_BUSY_avr --output-format csv -d $O/p3_$T -o run -- python3 bench/conv_once.py $S > $O/p3_$T.log 2>&1
done
