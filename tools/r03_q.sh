#!/bin/bash
set -u
export TMPDIR=/tmp
B=langsplatv2_amd/_build
V="base=langsplatv2_amd/liblsr.so m2=$B/var_m2/liblsr.so m4=$B/var_m4/liblsr.so m2r34=$B/var_m2r34/liblsr.so m4r17=$B/var_m4r17/liblsr.so m4r34=$B/var_m4r34/liblsr.so"
bash tools/r03_ab.sh r03q3 $V || exit 1
LSR_CFG=5 bash tools/r03_ab.sh r03q5 $V || exit 1
