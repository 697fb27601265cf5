#!/bin/bash
# A/B of liblsr variants in one process (tools/ab.py, cfg3 stage times) + the
# backward phase census of the stamps build.  Usage: bash tools/r04_ab.sh TAG name=path ...
set -u
TAG=$1; shift
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u tools/ab.py "$@" > gpurun_out/${TAG}_ab.txt 2>&1 || { echo "ab failed"; tail -20 gpurun_out/${TAG}_ab.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/${TAG}_ab.txt
if [ -f langsplatv2_amd/_build/var_stamps/liblsr.so ]; then
  timeout -k 10 200 python -u tools/bwd_stamps.py langsplatv2_amd/_build/var_stamps/liblsr.so > gpurun_out/${TAG}_stamps.txt 2>&1 || { echo "stamps failed"; tail -20 gpurun_out/${TAG}_stamps.txt; exit 1; }
  grep -v amdgpu.ids gpurun_out/${TAG}_stamps.txt
fi
