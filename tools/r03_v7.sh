#!/bin/bash
# Round-3 measurement pass v7: the
# full pass (GPU tests, PMC traffic, bench, rocprof, cfg5 bench) and the cfg4-shape feature-training step.
set -u
export TMPDIR=/tmp
B=langsplatv2_amd/_build
bash tools/r03_final.sh r03v7 || exit 1
timeout -k 10 300 python tools/bench_train_step.py > gpurun_out/r03v7_train_step.json 2> gpurun_out/r03v7_train_step.err || { echo "train step failed"; tail -20 gpurun_out/r03v7_train_step.err; exit 1; }
cat gpurun_out/r03v7_train_step.json
echo v7 done
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r03v7_smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/r03v7_smoke.log; exit 1; }
tail -2 gpurun_out/r03v7_smoke.log
