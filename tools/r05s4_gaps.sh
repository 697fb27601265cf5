#!/bin/bash
# Round-5 (session 4): per-dispatch gaps of the previous and the early-M
# builds (kernel trace of tools/ab.py with one library each), cfg3 and cfg2.
set -u
OUT=$(pwd)/gpurun_out; mkdir -p $OUT
ROOT=$(pwd)
cd /tmp && export TMPDIR=/tmp
for C in 3 2; do
for V in prev early; do
  L=$ROOT/langsplatv2_amd/liblsr.so; [ $V = prev ] && L=$ROOT/langsplatv2_amd/_build/var_prev/liblsr.so
  LSR_CFG=$C timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/r05s4_tr_${V}_$C -o run -- python3 $ROOT/tools/ab.py $V=$L > $OUT/r05s4_tr_${V}_$C.log 2>&1 || { echo "trace $V failed"; tail -20 $OUT/r05s4_tr_${V}_$C.log; exit 1; }
  CSV=$(find $OUT/r05s4_tr_${V}_$C -name "*kernel_trace.csv" | head -1)
  echo "== $V cfg$C"; tail -1 $OUT/r05s4_tr_${V}_$C.log
  python $ROOT/tools/gaps.py $CSV | grep "lsr::" | head -12
done
done
echo done
