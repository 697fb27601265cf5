#!/bin/bash
# SQ instruction/stall counters (two separate --pmc passes) over tools/pmc_step.py.
# Usage (repo root, on the GPU box): bash tools/pmc_sq.sh TAG [LIB]
set -e
TAG=$1; LIB=${2:-langsplatv2_amd/liblsr.so}
ROOT=$(pwd); OUT=$ROOT/gpurun_out/pmc_$TAG; mkdir -p $OUT; export TMPDIR=/tmp
case $LIB in /*) ;; *) LIB=$ROOT/$LIB;; esac
cd /tmp
P1="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_BRANCH"
P2="SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_WR"
LSR_LIB=$LIB LSR_STEPS=2 timeout -k 10 300 rocprofv3 --pmc $P1 -d $OUT/p1 -o run --output-format csv -- python3 $ROOT/tools/pmc_step.py > $OUT/p1.log 2>&1
LSR_LIB=$LIB LSR_STEPS=2 timeout -k 10 300 rocprofv3 --pmc $P2 -d $OUT/p2 -o run --output-format csv -- python3 $ROOT/tools/pmc_step.py > $OUT/p2.log 2>&1
echo "pmc $TAG done"
