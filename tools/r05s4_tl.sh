#!/bin/bash
# Round-5 (session 4): whole-step kernel traces (tools/pmc_step.py, no stage
# events) of the previous and the early-M builds at cfg3, binning timeline
# after the count; then bench.py with each library, both orders; the colour
# events with a device-scope release (evdev) A/B.
set -u
OUT=$(pwd)/gpurun_out; mkdir -p $OUT
ROOT=$(pwd)
PREV=$ROOT/langsplatv2_amd/_build/var_prev/liblsr.so
NEW=$ROOT/langsplatv2_amd/liblsr.so
EVD=$ROOT/langsplatv2_amd/_build/var_evdev/liblsr.so
cd /tmp && export TMPDIR=/tmp
for V in prev early evdev; do
  L=$NEW; [ $V = prev ] && L=$PREV; [ $V = evdev ] && L=$EVD
  LSR_LIB=$L LSR_STEPS=40 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/r05s4_tl_$V -o run -- python3 $ROOT/tools/pmc_step.py > $OUT/r05s4_tl_$V.log 2>&1 || { echo "trace $V failed"; tail -20 $OUT/r05s4_tl_$V.log; exit 1; }
  CSV=$(find $OUT/r05s4_tl_$V -name "*kernel_trace.csv" | head -1)
  echo "== $V"; python $ROOT/tools/timeline_bin.py $CSV; python $ROOT/tools/gaps.py $CSV | grep "lsr::" | head -4
done
cd $ROOT
for V in prev early early prev; do
  L=$NEW; [ $V = prev ] && L=$PREV
  LSR_LIB=$L timeout -k 10 300 python bench.py --no-cpu-baseline --no-fwd-1mpix > $OUT/r05s4_b_$V.json 2>/dev/null || { echo "bench $V failed"; exit 1; }
  echo "$V $(python -c "import json,sys; d=json.loads(open('$OUT/r05s4_b_$V.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])")"
done
LSR_LIB=$EVD timeout -k 10 300 python -u -m pytest tests/test_split_preprocess.py tests/test_view_stream.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/r05s4_evdev_tests.log 2>&1 || { echo "evdev tests failed"; tail -20 $OUT/r05s4_evdev_tests.log; exit 1; }
tail -1 $OUT/r05s4_evdev_tests.log
for C in 3 5; do
  LSR_CFG=$C timeout -k 10 300 python tools/ab.py early=$NEW evdev=$EVD > $OUT/r05s4_ab_evdev_cfg$C.txt 2>&1 || { echo "ab cfg$C failed"; exit 1; }
  LSR_CFG=$C timeout -k 10 300 python tools/ab.py evdev=$EVD early=$NEW > $OUT/r05s4_ab_evdev_rev_cfg$C.txt 2>&1 || { echo "ab rev cfg$C failed"; exit 1; }
  echo "== cfg$C"; tail -2 $OUT/r05s4_ab_evdev_cfg$C.txt; tail -2 $OUT/r05s4_ab_evdev_rev_cfg$C.txt
done
