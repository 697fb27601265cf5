#!/bin/bash
# LDS / scalar stall counters (two separate --pmc passes) over tools/pmc_step.py.
# Usage (repo root, on the GPU box): bash tools/pmc_stall.sh TAG
set -e
TAG=$1
ROOT=$(pwd); OUT=$ROOT/gpurun_out/pmc_$TAG; mkdir -p $OUT; export TMPDIR=/tmp
cd /tmp
P1="SQ_WAIT_INST_LDS SQ_INST_LEVEL_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_SCA SQ_LEVEL_WAVES"
P2="SQ_INSTS_LDS_LOAD_BANDWIDTH SQ_ACTIVE_INST_MISC SQ_INSTS_VALU_TRANS_F32 SQ_THREAD_CYCLES_VALU SQ_WAVES SQ_BUSY_CU_CYCLES SQ_CYCLES SQ_ACTIVE_INST_VALU2"
LSR_STEPS=2 timeout -s KILL 120 rocprofv3 --pmc $P1 -d $OUT/p1 -o run --output-format csv -- python3 $ROOT/tools/pmc_step.py > $OUT/p1.log 2>&1
LSR_STEPS=2 timeout -s KILL 120 rocprofv3 --pmc $P2 -d $OUT/p2 -o run --output-format csv -- python3 $ROOT/tools/pmc_step.py > $OUT/p2.log 2>&1
echo "pmc $TAG done"
