#!/bin/bash
set -u
export TMPDIR=/tmp
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r03_smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/r03_smoke.log; exit 1; }
tail -3 gpurun_out/r03_smoke.log
