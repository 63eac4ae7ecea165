# LDS counters of one 3x3 conv, current build vs an alternate build (arg 1)
set -e
O=gpurun_out/pmc_lds; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
S="320 64 64 32 3 1 1 20"
P="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL GRBM_GUI_ACTIVE"
timeout -k 10 120 rocprofv3 --pmc $P --output-format csv -d $O/new -o run -- python3 bench/conv_once.py $S > $O/new.log 2>&1
MERCURY_EXT_PATH=$1 timeout -k 10 120 rocprofv3 --pmc $P --output-format csv -d $O/old -o run -- python3 bench/conv_once.py $S > $O/old.log 2>&1
