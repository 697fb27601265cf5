#!/bin/bash
# Round-3 GPU pass: backward probe A/B (tools/ab.py), decode error, parity tests, cfg5 replica bench.
set -u
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
B=langsplatv2_amd/_build
timeout -k 10 300 python -u tools/ab.py base=langsplatv2_amd/liblsr.so nopro=$B/var_nopro/liblsr.so nofeat=$B/var_nofeat/liblsr.so noatom=$B/var_noatom/liblsr.so nomf=$B/var_nomf/liblsr.so > $OUT/r03a_ab.txt 2>&1 || { echo "ab failed"; tail -20 $OUT/r03a_ab.txt; exit 1; }
cat $OUT/r03a_ab.txt
timeout -k 10 300 python -u tools/dec_err.py > $OUT/r03a_dec_err.json 2>&1 || { echo "dec_err failed"; tail -20 $OUT/r03a_dec_err.json; exit 1; }
cat $OUT/r03a_dec_err.json
timeout -k 10 300 python -u bench.py --config 5 --steps 10 --warmup 3 > $OUT/r03a_cfg5.json 2> $OUT/r03a_cfg5.err || { echo "cfg5 bench failed"; tail -20 $OUT/r03a_cfg5.err; exit 1; }
cat $OUT/r03a_cfg5.json
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/r03a_gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -40 $OUT/r03a_gpu_tests.log; exit 1; }
tail -3 $OUT/r03a_gpu_tests.log
