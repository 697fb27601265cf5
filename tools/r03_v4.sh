#!/bin/bash
# Round-3 measurement pass v4: A/B of this build vs 76bfcc5's render (cfg3 at D = 16 and 64, cfg5), then the
# full pass (GPU tests, PMC traffic, bench, rocprof, cfg5 bench) and the cfg4-shape feature-training step.
set -u
export TMPDIR=/tmp
B=langsplatv2_amd/_build
bash tools/r03_ab.sh r03v4ab3 prev=$B/var_prev/liblsr.so now=langsplatv2_amd/liblsr.so || exit 1
LSR_D=64 bash tools/r03_ab.sh r03v4ab364 prev=$B/var_prev/liblsr.so now=langsplatv2_amd/liblsr.so || exit 1
LSR_CFG=5 bash tools/r03_ab.sh r03v4ab5 prev=$B/var_prev/liblsr.so now=langsplatv2_amd/liblsr.so || exit 1
bash tools/r03_final.sh r03v4 || exit 1
timeout -k 10 300 python tools/bench_train_step.py > gpurun_out/r03v4_train_step.json 2> gpurun_out/r03v4_train_step.err || { echo "train step failed"; tail -20 gpurun_out/r03v4_train_step.err; exit 1; }
cat gpurun_out/r03v4_train_step.json
echo v4 done
