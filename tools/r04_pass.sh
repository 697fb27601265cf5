#!/bin/bash
# Round-4 measurement pass on the GPU box (repo root, under gpurun):
#   1. pytest -m gpu (parity; stops at the first failure)
#   2. bench.py (the headline line) -> gpurun_out/${TAG}_bench.json
#   3. SQ counter passes (issue roofline) + FETCH/WRITE passes (HBM traffic) over tools/pmc_step.py
#   4. rocprofv3 --kernel-trace --stats of the bench
# Usage: bash tools/r04_pass.sh TAG [skip-tests]
set -u
TAG=${1:-r04a}
ROOT=$(pwd)
OUT=$ROOT/gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
if [ "${2:-}" != "skip-tests" ]; then
  # failures (exit 1) are reported and the pass goes on; a crash, abort or
  # time limit (any other status) ends it
  timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $OUT/${TAG}_gpu_tests.log 2>&1
  rc=$?
  grep -E "FAILED|passed|failed" $OUT/${TAG}_gpu_tests.log | tail -25
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "gpu tests ended with status $rc"; tail -30 $OUT/${TAG}_gpu_tests.log; exit 1; fi
fi
timeout -k 10 600 python bench.py > $OUT/${TAG}_bench.json 2> $OUT/${TAG}_bench.err || { echo "bench failed"; tail -20 $OUT/${TAG}_bench.err; exit 1; }
cat $OUT/${TAG}_bench.json
cd /tmp
P1="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_BRANCH"
P2="SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_WR"
LSR_STEPS=2 timeout -s KILL 120 rocprofv3 --pmc $P1 -d $OUT/${TAG}_sq1 -o run --output-format csv -- python3 $ROOT/tools/pmc_step.py > $OUT/${TAG}_sq1.log 2>&1 || { echo "sq1 failed"; exit 1; }
LSR_STEPS=2 timeout -s KILL 120 rocprofv3 --pmc $P2 -d $OUT/${TAG}_sq2 -o run --output-format csv -- python3 $ROOT/tools/pmc_step.py > $OUT/${TAG}_sq2.log 2>&1 || { echo "sq2 failed"; exit 1; }
LSR_STEPS=2 timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $OUT/${TAG}_pmcF -o run --output-format csv -- python3 $ROOT/tools/pmc_step.py > $OUT/${TAG}_pmcF.log 2>&1 || { echo "pmc fetch failed"; exit 1; }
LSR_STEPS=2 timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $OUT/${TAG}_pmcW -o run --output-format csv -- python3 $ROOT/tools/pmc_step.py > $OUT/${TAG}_pmcW.log 2>&1 || { echo "pmc write failed"; exit 1; }
cd $ROOT
python tools/pmc_issue.py $OUT/${TAG}_sq1 $OUT/${TAG}_sq2 $OUT/${TAG}_pmc_issue.json --units k_render_bwd_mf=3490000 > $OUT/${TAG}_pmc_issue.txt
python tools/pmc_traffic.py $OUT/${TAG}_pmcF $OUT/${TAG}_pmcW $OUT/${TAG}_pmc_traffic.json > $OUT/${TAG}_pmc_traffic.txt
cat $OUT/${TAG}_pmc_issue.txt
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/${TAG}_prof -o run -- python3 $ROOT/bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-fwd-1mpix > $OUT/${TAG}_prof.log 2>&1 || { echo "rocprof failed"; exit 1; }
cd $ROOT
DB=$(ls $OUT/${TAG}_prof/*/run_results.db $OUT/${TAG}_prof/run_results.db 2>/dev/null | head -1)
python tools/prof_summary.py $DB $OUT/${TAG}_kernel_stats.md "$TAG: bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-fwd-1mpix (cfg3) under rocprofv3 --kernel-trace --stats" > /dev/null || echo "summary failed"
echo "pass $TAG done"
