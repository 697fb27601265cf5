#!/bin/bash
set -u
export TMPDIR=/tmp
uptime
for k in 1 2; do timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/r03x_bench$k.json 2> gpurun_out/r03x_bench$k.err || { echo "bench failed"; tail -5 gpurun_out/r03x_bench$k.err; exit 1; }; python -c "import json;d=json.load(open('gpurun_out/r03x_bench$k.json'));print(d['value'],d['ms_per_step'],d['hbm_step'])"; done
uptime
