#!/bin/bash
# Round-5 (session 3): cfg3 binning: the count's block size and the chunk target, one-process A/B
# (two orders).
set -u
OUT=gpurun_out; mkdir -p $OUT
B=langsplatv2_amd/_build
LSR_CFG=3 timeout -k 10 600 python tools/ab.py c512=$B/var_c512/liblsr.so t768=$B/var_t768/liblsr.so c512t768=$B/var_c512t768/liblsr.so base=langsplatv2_amd/liblsr.so > $OUT/r05s3_ab_tune2_cfg3.txt 2>&1 || { echo "ab failed"; tail -20 $OUT/r05s3_ab_tune2_cfg3.txt; exit 1; }
cat $OUT/r05s3_ab_tune2_cfg3.txt
LSR_CFG=3 timeout -k 10 600 python tools/ab.py base=langsplatv2_amd/liblsr.so c512t768=$B/var_c512t768/liblsr.so t768=$B/var_t768/liblsr.so c512=$B/var_c512/liblsr.so > $OUT/r05s3_ab_tune3_cfg3.txt 2>&1 || { echo "ab failed"; tail -20 $OUT/r05s3_ab_tune3_cfg3.txt; exit 1; }
cat $OUT/r05s3_ab_tune3_cfg3.txt
echo done
