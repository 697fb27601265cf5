#!/bin/bash
# Round-5 (session 3): tile-count band height (34 / 68 / 135 rows), cfg5 and cfg3.
set -u
OUT=gpurun_out; mkdir -p $OUT
for C in 5 3; do
  LSR_CFG=$C timeout -k 10 500 python tools/ab.py base=langsplatv2_amd/liblsr.so c68=langsplatv2_amd/_build/var_c68/liblsr.so > $OUT/r05s3_ab_bands_cfg$C.txt 2>&1 || { echo "ab cfg$C failed"; tail -20 $OUT/r05s3_ab_bands_cfg$C.txt; exit 1; }
  cat $OUT/r05s3_ab_bands_cfg$C.txt
done
echo done
