set -u
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 120 python -u -m pytest tests/test_micro_checks.py -v -s --timeout 60 --timeout-method thread > $OUT/r05c_micro.log 2>&1; grep -E "max relative|passed|failed" $OUT/r05c_micro.log
timeout -k 10 120 python tools/fx_redo_count.py langsplatv2_amd/_build/var_fxmark/liblsr.so 3 5 2>&1 | tail -3
timeout -k 10 300 python tools/ab.py exact=langsplatv2_amd/_build/var_exact/liblsr.so fx=langsplatv2_amd/liblsr.so fxnr=langsplatv2_amd/_build/var_fxnr/liblsr.so > $OUT/r05c_ab.txt 2>&1; tail -20 $OUT/r05c_ab.txt
timeout -k 10 60 tools/micro/store_pattern > $OUT/r05c_store.txt 2>&1; cat $OUT/r05c_store.txt
