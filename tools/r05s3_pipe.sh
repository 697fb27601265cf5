#!/bin/bash
# Round-5 (session 3): the quick frame stream sequential vs pipelined over two
# streams, for several decode CU counts (tools/pipe_quick.py).
set -u
OUT=gpurun_out; mkdir -p $OUT
: > $OUT/r05s3_pipe.txt
for n in 255 192 128 96; do
  LSR_DEC_NCU=$n timeout -k 10 200 python tools/pipe_quick.py langsplatv2_amd/_build/var_decncu/liblsr.so >> $OUT/r05s3_pipe.txt 2>&1 || { echo "pipe $n failed"; tail -20 $OUT/r05s3_pipe.txt; exit 1; }
done
cat $OUT/r05s3_pipe.txt
echo done
