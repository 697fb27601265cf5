#!/bin/bash
set -u
export TMPDIR=/tmp
B=langsplatv2_amd/_build
bash tools/r03_ab.sh r03u3 base=langsplatv2_amd/liblsr.so she=$B/var_she/liblsr.so || exit 1
LSR_CFG=5 bash tools/r03_ab.sh r03u5 base=langsplatv2_amd/liblsr.so she=$B/var_she/liblsr.so || exit 1
