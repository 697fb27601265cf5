#!/bin/bash
# Round-5 (session 3): cfg5 binning tunables, one-process stage A/B (tools/ab.py).
set -u
OUT=gpurun_out; mkdir -p $OUT
LSR_CFG=5 timeout -k 10 500 python tools/ab.py base=langsplatv2_amd/liblsr.so m8=langsplatv2_amd/_build/var_m8/liblsr.so m2x=langsplatv2_amd/_build/var_m2x/liblsr.so s64=langsplatv2_amd/_build/var_s64/liblsr.so > $OUT/r05s3_cfg5_tunables.txt 2>&1 || { echo "ab failed"; tail -20 $OUT/r05s3_cfg5_tunables.txt; exit 1; }
cat $OUT/r05s3_cfg5_tunables.txt
echo done
