#!/bin/bash
# Round-5 (session 3): the colour stream's priority (lowest / highest / default), cfg3 and cfg5.
set -u
OUT=gpurun_out; mkdir -p $OUT
B=langsplatv2_amd/_build
for C in 3 5; do
  LSR_CFG=$C timeout -k 10 600 python tools/ab.py low=$B/var_lowprio/liblsr.so base=langsplatv2_amd/liblsr.so high=$B/var_hiprio/liblsr.so > $OUT/r05s3_ab_prio_cfg$C.txt 2>&1 || { echo "ab failed"; tail -20 $OUT/r05s3_ab_prio_cfg$C.txt; exit 1; }
  cat $OUT/r05s3_ab_prio_cfg$C.txt
done
echo done
