#!/bin/bash
# Round-5 (session 4): is the ~6 us gap before k_bin_scatter (its launch queued
# ~45 us ahead) tied to its > 64 KB LDS?  Whole-step traces of the shipped build
# and of 34-row scatter bands (50 KB LDS).
set -u
OUT=$(pwd)/gpurun_out; mkdir -p $OUT
ROOT=$(pwd)
cd /tmp && export TMPDIR=/tmp
for V in early sr34; do
  L=$ROOT/langsplatv2_amd/liblsr.so; [ $V = sr34 ] && L=$ROOT/langsplatv2_amd/_build/var_sr34/liblsr.so
  LSR_LIB=$L LSR_STEPS=30 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/r05s4_sg_$V -o run -- python3 $ROOT/tools/pmc_step.py > $OUT/r05s4_sg_$V.log 2>&1 || { echo "trace $V failed"; tail -20 $OUT/r05s4_sg_$V.log; exit 1; }
  CSV=$(find $OUT/r05s4_sg_$V -name "*kernel_trace.csv" | head -1)
  echo "== $V"; python $ROOT/tools/timeline_bin.py $CSV; python $ROOT/tools/gaps.py $CSV | grep "lsr::" | head -3
done
