#!/bin/bash
# One GPU-box pass: parity tests, PMC traffic passes, bench, kernel-trace profile.
# Usage (from the repo root, under gpurun): bash tools/gpu_round.sh TAG
set -u
TAG=${1:-r01}
ROOT=$(pwd)
OUT=$ROOT/gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -m gpu -x -q > $OUT/${TAG}_gpu_tests.log 2>&1 || { echo "gpu tests failed rc=$?"; tail -30 $OUT/${TAG}_gpu_tests.log; exit 1; }
tail -3 $OUT/${TAG}_gpu_tests.log
cd /tmp
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/${TAG}_pmcF -o run --output-format csv -- python3 $ROOT/tools/pmc_step.py > $OUT/${TAG}_pmcF.log 2>&1 || { echo "pmc fetch failed"; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/${TAG}_pmcW -o run --output-format csv -- python3 $ROOT/tools/pmc_step.py > $OUT/${TAG}_pmcW.log 2>&1 || { echo "pmc write failed"; exit 1; }
cd $ROOT
python tools/pmc_traffic.py $OUT/${TAG}_pmcF $OUT/${TAG}_pmcW profiles/${TAG}_pmc_traffic.json > $OUT/${TAG}_pmc_traffic.txt && cp profiles/${TAG}_pmc_traffic.json $OUT/
timeout -k 10 900 python bench.py > $OUT/${TAG}_bench.json 2> $OUT/${TAG}_bench.err || { echo "bench failed"; tail -20 $OUT/${TAG}_bench.err; exit 1; }
cat $OUT/${TAG}_bench.json
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/${TAG}_prof -o run -- python3 $ROOT/bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-fwd-1mpix > $OUT/${TAG}_prof.log 2>&1 || { echo "rocprof failed"; exit 1; }
echo done
