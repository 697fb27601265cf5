#!/bin/bash
# A/B of liblsr variants in one process (tools/ab.py), cfg3 (or LSR_CFG).
# Usage: bash tools/r05_ab.sh TAG name=path.so ...
set -u
TAG=$1; shift
mkdir -p gpurun_out
timeout -k 10 300 python tools/ab.py "$@" > gpurun_out/${TAG}_ab.txt 2>&1 || { echo "ab failed"; tail -20 gpurun_out/${TAG}_ab.txt; exit 1; }
tail -12 gpurun_out/${TAG}_ab.txt
