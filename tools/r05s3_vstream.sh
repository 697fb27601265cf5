#!/bin/bash
# Round-5 (session 3): ViewStream tests, then the cfg5 and cfg2 lines with view_stream_fps.
set -u
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_view_stream.py tests/test_quick_stream.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/r05s3_vstream_tests.log 2>&1 || { echo "tests failed"; tail -30 $OUT/r05s3_vstream_tests.log; exit 1; }
tail -1 $OUT/r05s3_vstream_tests.log
for C in 5 2; do
  timeout -k 10 500 python bench.py --config $C --no-cpu-baseline > $OUT/r05s3_vstream_cfg$C.json 2> $OUT/r05s3_vstream_cfg$C.err || { echo "bench cfg$C failed"; tail -20 $OUT/r05s3_vstream_cfg$C.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/r05s3_vstream_cfg$C.json')); print('cfg$C', d['value'], d['view_stream_fps'])"
done

timeout -k 10 500 python bench.py --no-cpu-baseline --no-fwd-1mpix > $OUT/r05s3_vstream_cfg3.json 2> $OUT/r05s3_vstream_cfg3.err || { echo "bench cfg3 failed"; tail -20 $OUT/r05s3_vstream_cfg3.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/r05s3_vstream_cfg3.json')); print('cfg3', d['value'], d['quick_1mpix'])"
echo done
