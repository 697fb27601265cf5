#!/bin/bash
# Round-5 (session 2) quick-path probes on the GPU box: store patterns, the
# decode's store-layout A/B, then the r05 pass steps given as $1.
set -u
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 120 tools/micro/store_pattern > $OUT/r05s2_store_patterns.txt 2>&1 || { echo "store probe failed"; cat $OUT/r05s2_store_patterns.txt; exit 1; }
cat $OUT/r05s2_store_patterns.txt
timeout -k 10 300 python -u -m pytest tests/test_quick_decode.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/r05s2_qdec_tests.log 2>&1 || { echo "quick decode tests failed"; tail -30 $OUT/r05s2_qdec_tests.log; exit 1; }
tail -2 $OUT/r05s2_qdec_tests.log
timeout -k 10 300 python tools/ab_quick.py head=langsplatv2_amd/_build/var_head/liblsr.so decA=langsplatv2_amd/_build/var_decA/liblsr.so new=langsplatv2_amd/liblsr.so > $OUT/r05s2_ab_quick_store.txt 2>&1 || { echo "ab_quick failed"; tail -20 $OUT/r05s2_ab_quick_store.txt; exit 1; }
cat $OUT/r05s2_ab_quick_store.txt
[ -n "${1:-}" ] && bash tools/r05_pass.sh r05s2a "$1"
echo done
