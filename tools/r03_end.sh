#!/bin/bash
# Round-3 end check on the committed build: smoke(), then the default bench line.
set -u
export TMPDIR=/tmp
OUT=gpurun_out
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/r03end_smoke.log 2>&1 || { echo "smoke failed"; tail -20 $OUT/r03end_smoke.log; exit 1; }
tail -2 $OUT/r03end_smoke.log
timeout -k 10 600 python bench.py > $OUT/r03end_bench.json 2> $OUT/r03end_bench.err || { echo "bench failed"; tail -20 $OUT/r03end_bench.err; exit 1; }
cat $OUT/r03end_bench.json
