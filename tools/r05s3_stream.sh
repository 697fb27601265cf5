#!/bin/bash
# Round-5 (session 3): the streamed quick path: its GPU tests, then the bench line.
set -u
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_quick_stream.py tests/test_quick_packed.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/r05s3_stream_tests.log 2>&1 || { echo "stream tests failed"; tail -30 $OUT/r05s3_stream_tests.log; exit 1; }
tail -2 $OUT/r05s3_stream_tests.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/r05s3_bench.json 2> $OUT/r05s3_bench.err || { echo "bench failed"; tail -20 $OUT/r05s3_bench.err; exit 1; }
cat $OUT/r05s3_bench.json
echo done
