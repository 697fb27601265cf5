#!/bin/bash
# Round-5 (session 4): does the runtime hold the scatter's dispatch until the
# next launch?  Whole-step traces (pmc_step.py) with and without a
# hipStreamQuery right after the scatter launch, then tools/ab.py + bench.py.
set -u
OUT=$(pwd)/gpurun_out; mkdir -p $OUT
ROOT=$(pwd)
NEW=$ROOT/langsplatv2_amd/liblsr.so
FL=$ROOT/langsplatv2_amd/_build/var_flush/liblsr.so
cd /tmp && export TMPDIR=/tmp
for V in early flush; do
  L=$NEW; [ $V = flush ] && L=$FL
  LSR_LIB=$L LSR_STEPS=30 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/r05s4_fl_$V -o run -- python3 $ROOT/tools/pmc_step.py > $OUT/r05s4_fl_$V.log 2>&1 || { echo "trace $V failed"; tail -20 $OUT/r05s4_fl_$V.log; exit 1; }
  CSV=$(find $OUT/r05s4_fl_$V -name "*kernel_trace.csv" | head -1)
  echo "== $V"; python $ROOT/tools/timeline_bin.py $CSV; python $ROOT/tools/gaps.py $CSV | grep "lsr::" | head -3
done
cd $ROOT
for C in 3 5 2; do
  LSR_CFG=$C timeout -k 10 300 python tools/ab.py early=$NEW flush=$FL > $OUT/r05s4_ab_flush_cfg$C.txt 2>&1 || { echo "ab cfg$C failed"; exit 1; }
  LSR_CFG=$C timeout -k 10 300 python tools/ab.py flush=$FL early=$NEW > $OUT/r05s4_ab_flush_rev_cfg$C.txt 2>&1 || { echo "ab rev cfg$C failed"; exit 1; }
  echo "== cfg$C"; tail -2 $OUT/r05s4_ab_flush_cfg$C.txt | sed 's/.*SUM/SUM/'; tail -2 $OUT/r05s4_ab_flush_rev_cfg$C.txt | sed 's/.*SUM/SUM/'
done
for V in early flush flush early; do
  L=$NEW; [ $V = flush ] && L=$FL
  LSR_LIB=$L timeout -k 10 300 python bench.py --no-cpu-baseline --no-fwd-1mpix > $OUT/r05s4_fb_$V.json 2>/dev/null || { echo "bench $V failed"; exit 1; }
  echo "$V $(python -c "import json; d=json.loads(open('$OUT/r05s4_fb_$V.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])")"
done
