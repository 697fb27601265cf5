#!/bin/bash
# forward GEO4 staging: GPU tests, A/B vs GEO4=0, LDS-activity PMC pass on the render kernels.
set -u
export TMPDIR=/tmp
B=langsplatv2_amd/_build
ROOT=$(pwd); OUT=$ROOT/gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/r03geo_gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -40 $OUT/r03geo_gpu_tests.log; exit 1; }
tail -2 $OUT/r03geo_gpu_tests.log
bash tools/r03_ab.sh r03geo3 geo0=$B/var_geo0/liblsr.so geo4=langsplatv2_amd/liblsr.so || exit 1
LSR_CFG=5 bash tools/r03_ab.sh r03geo5 geo0=$B/var_geo0/liblsr.so geo4=langsplatv2_amd/liblsr.so || exit 1
cd /tmp
LSR_STEPS=2 timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_ACTIVE_INST_VALU -d $OUT/r03geo_lds -o run --output-format csv -- python3 $ROOT/tools/pmc_step.py > $OUT/r03geo_lds.log 2>&1 || { echo "pmc failed"; tail -5 $OUT/r03geo_lds.log; exit 1; }
cd $ROOT
python tools/pmc_kernel.py $OUT/r03geo_lds k_render_fwd $OUT/r03geo_lds k_render_bwd > $OUT/r03geo_lds.txt && cat $OUT/r03geo_lds.txt
echo done
