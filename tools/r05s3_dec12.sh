#!/bin/bash
# Round-5 (session 3): the decode with 12 waves per workgroup (3 per SIMD, no weight prefetch)
# and with 8 waves without the prefetch, against the build; hwc and chw maps.
set -u
OUT=gpurun_out; mkdir -p $OUT
B=langsplatv2_amd/_build
for L in hwc chw; do
  LSR_AB_LAYOUT=$L timeout -k 10 300 python tools/ab_quick.py base=langsplatv2_amd/liblsr.so dec12=$B/var_dec12/liblsr.so dec8np=$B/var_dec8np/liblsr.so > $OUT/r05s3_ab_dec12_$L.txt 2>&1 || { echo "ab_quick failed"; tail -20 $OUT/r05s3_ab_dec12_$L.txt; exit 1; }
  cat $OUT/r05s3_ab_dec12_$L.txt
done
echo done
