#!/bin/bash
# Round-5 (session 3): render tile order band height, one-wave tile sort size and
# the table scan's rows per thread, cfg3 and cfg5 (base = the previous build).
set -u
OUT=gpurun_out; mkdir -p $OUT
B=langsplatv2_amd/_build
for C in 3 5; do
  LSR_CFG=$C timeout -k 10 600 python tools/ab.py band2=$B/var_band2/liblsr.so base=$B/var_prev/liblsr.so tbl8=langsplatv2_amd/liblsr.so band8=$B/var_band8/liblsr.so swm2048=$B/var_swm2048/liblsr.so > $OUT/r05s3_ab_tune4_cfg$C.txt 2>&1 || { echo "ab failed"; tail -20 $OUT/r05s3_ab_tune4_cfg$C.txt; exit 1; }
  cat $OUT/r05s3_ab_tune4_cfg$C.txt
done
echo done
