#!/bin/bash
# PMC passes over the quick path (tools/pmc_step.py LSR_QUICK=1: quick render + codebook decode at
# 1280x800, 1M Gaussians): HBM traffic (FETCH_SIZE, WRITE_SIZE) and SQ instruction/busy counters,
# each in its own rocprofv3 pass.  Usage (repo root, GPU box): bash tools/pmc_quick.sh TAG
set -u
TAG=$1
ROOT=$(pwd); OUT=$ROOT/gpurun_out/pmcq_$TAG; mkdir -p $OUT; export TMPDIR=/tmp
cd /tmp
run() {  # name, counters
    LSR_QUICK=1 LSR_STEPS=2 timeout -s KILL 120 rocprofv3 --pmc $2 -d $OUT/$1 -o run --output-format csv -- python3 $ROOT/tools/pmc_step.py > $OUT/$1.log 2>&1 || { echo "pmc pass $1 failed"; tail -5 $OUT/$1.log; exit 1; }
}
run F "FETCH_SIZE"
run W "WRITE_SIZE"
run S1 "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_BRANCH"
run S2 "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_WR"
cd $ROOT
python tools/pmc_traffic.py $OUT/F $OUT/W $OUT/quick_traffic.json > $OUT/traffic.txt && cat $OUT/traffic.txt
python tools/pmc_kernel.py $OUT/S1 k_render_fwd_quick_d $OUT/S2 k_render_fwd_quick_d $OUT/S1 k_quick_decode_l $OUT/S2 k_quick_decode_l > $OUT/sq.txt 2>&1; cat $OUT/sq.txt
echo "pmc quick $TAG done"
