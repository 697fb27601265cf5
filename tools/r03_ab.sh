#!/bin/bash
# A/B of render variants in one process (tools/ab.py). Usage: bash tools/r03_ab.sh TAG name=path ...
set -u
TAG=$1; shift
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/ab.py "$@" > gpurun_out/${TAG}_ab.txt 2>&1 || { echo "ab failed"; tail -20 gpurun_out/${TAG}_ab.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/${TAG}_ab.txt
