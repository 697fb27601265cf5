#!/bin/bash
# render_bwd moments from column-parity sums (var_mom): GPU tests on it, A/B vs the product (cfg3 at D = 16 and 64);
# cfg5 PMC traffic passes (FETCH_SIZE / WRITE_SIZE) for bench.py's cfg5 line.
set -u
export TMPDIR=/tmp
B=langsplatv2_amd/_build
ROOT=$(pwd); OUT=$ROOT/gpurun_out
cp langsplatv2_amd/liblsr.so $B/prod.so
cd /tmp
LSR_CFG=5 LSR_STEPS=2 timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/cfg5_r03v4_pmcF -o run --output-format csv -- python3 $ROOT/tools/pmc_step.py > $OUT/cfg5_r03v4_pmcF.log 2>&1 || { echo "pmc fetch failed"; exit 1; }
LSR_CFG=5 LSR_STEPS=2 timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/cfg5_r03v4_pmcW -o run --output-format csv -- python3 $ROOT/tools/pmc_step.py > $OUT/cfg5_r03v4_pmcW.log 2>&1 || { echo "pmc write failed"; exit 1; }
cd $ROOT
python tools/pmc_traffic.py $OUT/cfg5_r03v4_pmcF $OUT/cfg5_r03v4_pmcW $OUT/cfg5_r03v4_pmc_traffic.json > $OUT/cfg5_r03v4_pmc_traffic.txt && cat $OUT/cfg5_r03v4_pmc_traffic.txt | head -8
cp $B/var_mom/liblsr.so langsplatv2_amd/liblsr.so
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/r03mom_gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -40 $OUT/r03mom_gpu_tests.log; exit 1; }
tail -2 $OUT/r03mom_gpu_tests.log
bash tools/r03_ab.sh r03mom3 prod=$B/prod.so mom=$B/var_mom/liblsr.so || exit 1
LSR_D=64 bash tools/r03_ab.sh r03mom364 prod=$B/prod.so mom=$B/var_mom/liblsr.so || exit 1
echo done
