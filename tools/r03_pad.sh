#!/bin/bash
# forward: padding channel not accumulated (pad) vs HEAD render (pad0): A/B cfg3 + cfg5; SQ issue counters on the product build.
set -u
export TMPDIR=/tmp
B=langsplatv2_amd/_build
ROOT=$(pwd); OUT=$ROOT/gpurun_out
bash tools/r03_ab.sh r03pad3 pad0=$B/var_pad0/liblsr.so pad=langsplatv2_amd/liblsr.so || exit 1
LSR_CFG=5 bash tools/r03_ab.sh r03pad5 pad0=$B/var_pad0/liblsr.so pad=langsplatv2_amd/liblsr.so || exit 1
cd /tmp
LSR_STEPS=2 timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_MFMA -d $OUT/r03v3_sq1 -o run --output-format csv -- python3 $ROOT/tools/pmc_step.py > $OUT/r03v3_sq1.log 2>&1 || { echo "pmc1 failed"; tail -5 $OUT/r03v3_sq1.log; exit 1; }
LSR_STEPS=2 timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_SALU SQ_ACTIVE_INST_SCA -d $OUT/r03v3_sq2 -o run --output-format csv -- python3 $ROOT/tools/pmc_step.py > $OUT/r03v3_sq2.log 2>&1 || { echo "pmc2 failed"; tail -5 $OUT/r03v3_sq2.log; exit 1; }
cd $ROOT
python tools/pmc_kernel.py $OUT/r03v3_sq1 k_render_fwd $OUT/r03v3_sq1 k_render_bwd $OUT/r03v3_sq2 k_render_fwd $OUT/r03v3_sq2 k_render_bwd > $OUT/r03v3_sq.txt && cat $OUT/r03v3_sq.txt
echo done
