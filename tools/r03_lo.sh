#!/bin/bash
# language-only backward with atomics straight from the MFMA accumulators: GPU tests, then the cfg4-shape
# training step (D = 64, language-only backward) on the old (lo0) and new library, alternated.
set -u
export TMPDIR=/tmp
B=langsplatv2_amd/_build
OUT=gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/r03lo_gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -40 $OUT/r03lo_gpu_tests.log; exit 1; }
tail -2 $OUT/r03lo_gpu_tests.log
for i in 1 2; do
  LSR_LIB=$B/var_lo0/liblsr.so timeout -k 10 300 python tools/bench_train_step.py > $OUT/r03lo_old$i.json 2> $OUT/r03lo_old$i.err || { echo "old failed"; tail -5 $OUT/r03lo_old$i.err; exit 1; }
  timeout -k 10 300 python tools/bench_train_step.py > $OUT/r03lo_new$i.json 2> $OUT/r03lo_new$i.err || { echo "new failed"; tail -5 $OUT/r03lo_new$i.err; exit 1; }
  echo "old: $(cat $OUT/r03lo_old$i.json | python -c 'import json,sys; d=json.load(sys.stdin); print(d["ms_per_iteration"], d["rasterizer_stages_ms"]["render_bwd"])')"
  echo "new: $(cat $OUT/r03lo_new$i.json | python -c 'import json,sys; d=json.load(sys.stdin); print(d["ms_per_iteration"], d["rasterizer_stages_ms"]["render_bwd"])')"
done
echo done
