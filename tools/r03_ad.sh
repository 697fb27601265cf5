#!/bin/bash
set -u
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/bwd_stamps.py > gpurun_out/r03ad_stamps.txt 2>&1 || { echo "stamps failed"; tail -20 gpurun_out/r03ad_stamps.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/r03ad_stamps.txt
