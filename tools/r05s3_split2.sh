#!/bin/bash
# Round-5 (session 3): split preprocess at its 2M threshold: tests, GPU suite, cfg5 bench line.
set -u
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_split_preprocess.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/r05s3_split_tests.log 2>&1 || { echo "split tests failed"; tail -30 $OUT/r05s3_split_tests.log; exit 1; }
tail -2 $OUT/r05s3_split_tests.log
bash tools/r05_pass.sh r05s3d "tests cfg5" || exit 1
echo done
