#!/bin/bash
set -u
export TMPDIR=/tmp
ROOT=$(pwd); OUT=$ROOT/gpurun_out; B=$ROOT/langsplatv2_amd/_build
cd /tmp
LSR_LIB=$B/var_stg/liblsr.so LSR_STEPS=2 timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $OUT/r03ab2_W -o run --output-format csv -- python3 $ROOT/tools/pmc_step.py > $OUT/r03ab2_W.log 2>&1 || { echo "pmc failed"; tail -5 $OUT/r03ab2_W.log; exit 1; }
LSR_LIB=$B/var_stg/liblsr.so LSR_STEPS=2 timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $OUT/r03ab2_F -o run --output-format csv -- python3 $ROOT/tools/pmc_step.py > $OUT/r03ab2_F.log 2>&1 || { echo "pmc failed"; tail -5 $OUT/r03ab2_F.log; exit 1; }
cd $ROOT
python tools/pmc_traffic.py $OUT/r03ab2_F $OUT/r03ab2_W $OUT/r03ab2_traffic.json > $OUT/r03ab2_traffic.txt; grep -i scatter $OUT/r03ab2_traffic.txt
