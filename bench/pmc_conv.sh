set -e
mkdir -p gpurun_out/pmc2
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
S="320 64 64 32 3 1 1 20"
timeout -k 10 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_BUSY_CYCLES --output-format csv -d gpurun_out/pmc2/p1 -o run -- python3 bench/conv_once.py $S > gpurun_out/pmc2/p1.log 2>&1
timeout -k 10 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmc2/p2 -o run -- python3 bench/conv_once.py $S > gpurun_out/pmc2/p2.log 2>&1
timeout -k 10 120 rocprofv3 --pmc TA_BUSY_avr TCP_TOTAL_CACHE_ACCESSES_sum TCC_HIT_sum TCC_MISS_sum SQ_INSTS_SALU SQ_INSTS_SMEM --output-format csv -d gpurun_out/pmc2/p3 -o run -- python3 bench/conv_once.py $S > gpurun_out/pmc2/p3.log 2>&1 || true
