#!/bin/bash
# Round-5 measurement pass on the GPU box (repo root, under gpurun).
# Usage: bash tools/r05_pass.sh TAG "STEPS"
#   STEPS (space separated, run in this order, default "tests bench"):
#     tests   pytest -m gpu (all; failures reported, a crash/abort/time limit ends the pass)
#     ftests  pytest tests/test_fullsize.py only
#     bench   python bench.py (the headline line) -> gpurun_out/TAG_bench.json
#     cfg1 / cfg2 / cfg5   bench.py --config N lines -> gpurun_out/TAG_cfgN.json
#     pmc     SQ issue passes + FETCH/WRITE traffic passes over tools/pmc_step.py (cfg3)
#     pmc2 / pmc5  FETCH/WRITE traffic passes at cfg2 / cfg5 (LSR_CFG=N)
#     prof    rocprofv3 --kernel-trace --stats of bench.py (cfg3)
set -u
TAG=${1:-r05a}
STEPS=${2:-"tests bench"}
ROOT=$(pwd)
OUT=$ROOT/gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
for S in $STEPS; do
  echo "== $S"
  case $S in
  tests|ftests)
    T=tests; [ $S = ftests ] && T=tests/test_fullsize.py
    timeout -k 10 1000 python -u -m pytest $T -m gpu -v --timeout 400 --timeout-method thread --durations=20 > $OUT/${TAG}_${S}.log 2>&1
    rc=$?
    grep -E "FAILED|passed|failed" $OUT/${TAG}_${S}.log | tail -25
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "gpu tests ended with status $rc"; tail -30 $OUT/${TAG}_${S}.log; exit 1; fi
    ;;
  bench)
    timeout -k 10 600 python bench.py > $OUT/${TAG}_bench.json 2> $OUT/${TAG}_bench.err || { echo "bench failed"; tail -20 $OUT/${TAG}_bench.err; exit 1; }
    cat $OUT/${TAG}_bench.json
    ;;
  cfg1|cfg2|cfg5)
    N=${S#cfg}
    timeout -k 10 600 python bench.py --config $N > $OUT/${TAG}_$S.json 2> $OUT/${TAG}_$S.err || { echo "bench $S failed"; tail -20 $OUT/${TAG}_$S.err; exit 1; }
    cat $OUT/${TAG}_$S.json
    ;;
  pmc)
    cd /tmp
    P1="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_BRANCH"
    P2="SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_WR"
    LSR_STEPS=2 timeout -s KILL 120 rocprofv3 --pmc $P1 -d $OUT/${TAG}_sq1 -o run --output-format csv -- python3 $ROOT/tools/pmc_step.py > $OUT/${TAG}_sq1.log 2>&1 || { echo "sq1 failed"; exit 1; }
    LSR_STEPS=2 timeout -s KILL 120 rocprofv3 --pmc $P2 -d $OUT/${TAG}_sq2 -o run --output-format csv -- python3 $ROOT/tools/pmc_step.py > $OUT/${TAG}_sq2.log 2>&1 || { echo "sq2 failed"; exit 1; }
    LSR_STEPS=2 timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $OUT/${TAG}_pmcF -o run --output-format csv -- python3 $ROOT/tools/pmc_step.py > $OUT/${TAG}_pmcF.log 2>&1 || { echo "pmc fetch failed"; exit 1; }
    LSR_STEPS=2 timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $OUT/${TAG}_pmcW -o run --output-format csv -- python3 $ROOT/tools/pmc_step.py > $OUT/${TAG}_pmcW.log 2>&1 || { echo "pmc write failed"; exit 1; }
    cd $ROOT
    UNITS=$(python tools/lst_units.py 2>/dev/null || echo 3490000)
    python tools/pmc_issue.py $OUT/${TAG}_sq1 $OUT/${TAG}_sq2 $OUT/${TAG}_pmc_issue.json --units k_render_bwd_mf=$UNITS > $OUT/${TAG}_pmc_issue.txt
    python tools/pmc_traffic.py $OUT/${TAG}_pmcF $OUT/${TAG}_pmcW $OUT/${TAG}_pmc_traffic.json > $OUT/${TAG}_pmc_traffic.txt
    cat $OUT/${TAG}_pmc_issue.txt $OUT/${TAG}_pmc_traffic.txt
    ;;
  pmc2|pmc5)
    N=${S#pmc}
    cd /tmp
    LSR_CFG=$N LSR_STEPS=2 timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE -d $OUT/${TAG}_c${N}F -o run --output-format csv -- python3 $ROOT/tools/pmc_step.py > $OUT/${TAG}_c${N}F.log 2>&1 || { echo "pmc fetch cfg$N failed"; exit 1; }
    LSR_CFG=$N LSR_STEPS=2 timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE -d $OUT/${TAG}_c${N}W -o run --output-format csv -- python3 $ROOT/tools/pmc_step.py > $OUT/${TAG}_c${N}W.log 2>&1 || { echo "pmc write cfg$N failed"; exit 1; }
    cd $ROOT
    python tools/pmc_traffic.py $OUT/${TAG}_c${N}F $OUT/${TAG}_c${N}W $OUT/cfg${N}_${TAG}_pmc_traffic.json > $OUT/cfg${N}_${TAG}_pmc_traffic.txt
    cat $OUT/cfg${N}_${TAG}_pmc_traffic.txt
    ;;
  prof)
    cd /tmp
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/${TAG}_prof -o run -- python3 $ROOT/bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-fwd-1mpix > $OUT/${TAG}_prof.log 2>&1 || { echo "rocprof failed"; exit 1; }
    cd $ROOT
    DB=$(ls $OUT/${TAG}_prof/*/run_results.db $OUT/${TAG}_prof/run_results.db 2>/dev/null | head -1)
    python tools/prof_summary.py $DB $OUT/${TAG}_kernel_stats.md "$TAG: bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-fwd-1mpix (cfg3) under rocprofv3 --kernel-trace --stats" > /dev/null || echo "summary failed"
    head -30 $OUT/${TAG}_kernel_stats.md
    ;;
  *) echo "unknown step $S"; exit 1;;
  esac
done
echo "pass $TAG done"
