#!/bin/bash
# Re-entry check: GPU tests + smoke + bench on the current HEAD.
set -u
export TMPDIR=/tmp
OUT=gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/r03h_gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -30 $OUT/r03h_gpu_tests.log; exit 1; }
tail -2 $OUT/r03h_gpu_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/r03h_smoke.log 2>&1 || { echo "smoke failed"; tail -20 $OUT/r03h_smoke.log; exit 1; }
timeout -k 10 600 python bench.py > $OUT/r03h_bench.json 2> $OUT/r03h_bench.err || { echo "bench failed"; tail -20 $OUT/r03h_bench.err; exit 1; }
cat $OUT/r03h_bench.json
