#!/bin/bash
# Round-5 (session 3): per-dispatch gaps of a cfg3 step with the split preprocess on / off.
set -u
OUT=$(pwd)/gpurun_out; mkdir -p $OUT
ROOT=$(pwd)
cd /tmp && export TMPDIR=/tmp
for V in fused split; do
  L=$ROOT/langsplatv2_amd/liblsr.so; [ $V = fused ] && L="$L#split0"
  LSR_CFG=3 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/r05s3_g2_$V -o run -- python3 $ROOT/tools/ab.py $V=$L > $OUT/r05s3_g2_$V.log 2>&1 || { echo "trace $V failed"; tail -20 $OUT/r05s3_g2_$V.log; exit 1; }
  CSV=$(find $OUT/r05s3_g2_$V -name "*kernel_trace.csv" | head -1)
  echo "== $V"; python $ROOT/tools/gaps.py $CSV | grep "lsr::" | head -12
done
echo done
