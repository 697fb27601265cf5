#!/bin/bash
# Round-5 (session 3): per-dispatch kernel trace of the cfg3 bench step (gaps between kernels).
set -u
OUT=$(pwd)/gpurun_out; mkdir -p $OUT
ROOT=$(pwd)
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/r05s3_trace -o run -- python3 $ROOT/bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-fwd-1mpix --no-quick > $OUT/r05s3_trace.log 2>&1 || { echo "trace failed"; tail -20 $OUT/r05s3_trace.log; exit 1; }
cd $ROOT
CSV=$(find $OUT/r05s3_trace -name "*kernel_trace.csv" | head -1)
python tools/gaps.py $CSV > $OUT/r05s3_gaps.txt
head -30 $OUT/r05s3_gaps.txt
echo done
