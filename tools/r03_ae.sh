#!/bin/bash
set -u
export TMPDIR=/tmp
ROOT=$(pwd); OUT=$ROOT/gpurun_out
cd /tmp
LSR_CFG=5 LSR_STEPS=2 timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE -d $OUT/r03ae_W -o run --output-format csv -- python3 $ROOT/tools/pmc_step.py > $OUT/r03ae_W.log 2>&1 || { echo "pmc W failed"; tail -5 $OUT/r03ae_W.log; exit 1; }
LSR_CFG=5 LSR_STEPS=2 timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -d $OUT/r03ae_F -o run --output-format csv -- python3 $ROOT/tools/pmc_step.py > $OUT/r03ae_F.log 2>&1 || { echo "pmc F failed"; tail -5 $OUT/r03ae_F.log; exit 1; }
cd $ROOT
python tools/pmc_traffic.py $OUT/r03ae_F $OUT/r03ae_W $OUT/r03ae_cfg5_pmc_traffic.json > $OUT/r03ae_cfg5_pmc_traffic.txt; cat $OUT/r03ae_cfg5_pmc_traffic.txt
