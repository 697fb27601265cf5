#!/bin/bash
# Round-3 measurement pass: GPU tests, PMC traffic, bench (cfg3), rocprof, bench --config 5.
set -u
export TMPDIR=/tmp
T=${1:-r03v1}
bash tools/gpu_round.sh $T || exit 1
timeout -k 10 600 python bench.py --config 5 > gpurun_out/${T}_cfg5.json 2> gpurun_out/${T}_cfg5.err || { echo "cfg5 bench failed"; tail -20 gpurun_out/${T}_cfg5.err; exit 1; }
cat gpurun_out/${T}_cfg5.json
python tools/prof_summary.py gpurun_out/${T}_prof/run_results.db gpurun_out/${T}_kernel_stats.md "$T: bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-fwd-1mpix (cfg3) under rocprofv3 --kernel-trace --stats" > /dev/null
echo final done
