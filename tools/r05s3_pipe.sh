#!/bin/bash
# Round-5 (session 3): the quick frame stream: sequential, pipelined over two
# side streams, and quick.QuickFeatureStream from the default / a side stream.
set -u
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 200 python tools/pipe_quick.py > $OUT/r05s3_pipe2.txt 2>&1 || { echo "pipe failed"; tail -20 $OUT/r05s3_pipe2.txt; exit 1; }
cat $OUT/r05s3_pipe2.txt
echo done
