#!/bin/bash
# Round-5 (session 3): where the split preprocess's colour pass starts (behind
# the geometry / behind the tile count) and from which size, cfg3 and cfg5.
set -u
OUT=gpurun_out; mkdir -p $OUT
for C in 3 5; do
  LSR_CFG=$C timeout -k 10 500 python tools/ab.py fused=langsplatv2_amd/liblsr.so#split0 prod=langsplatv2_amd/liblsr.so sgc=langsplatv2_amd/_build/var_sgc/liblsr.so sac=langsplatv2_amd/_build/var_sac/liblsr.so > $OUT/r05s3_ab_split_start_cfg$C.txt 2>&1 || { echo "ab cfg$C failed"; tail -20 $OUT/r05s3_ab_split_start_cfg$C.txt; exit 1; }
  cat $OUT/r05s3_ab_split_start_cfg$C.txt
done
echo done
