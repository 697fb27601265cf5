set -u
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp; cd /tmp
P1="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_BRANCH"
P2="SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_WR"
LSR_CFG=5 LSR_STEPS=2 timeout -s KILL 120 rocprofv3 --pmc $P1 -d $OUT/c5_sq1 -o run --output-format csv -- python3 $ROOT/tools/pmc_step.py > $OUT/c5_sq1.log 2>&1 || { echo sq1 failed; exit 1; }
LSR_CFG=5 LSR_STEPS=2 timeout -s KILL 120 rocprofv3 --pmc $P2 -d $OUT/c5_sq2 -o run --output-format csv -- python3 $ROOT/tools/pmc_step.py > $OUT/c5_sq2.log 2>&1 || { echo sq2 failed; exit 1; }
LSR_CFG=5 LSR_STEPS=2 timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $OUT/c5_F -o run --output-format csv -- python3 $ROOT/tools/pmc_step.py > $OUT/c5_F.log 2>&1 || { echo F failed; exit 1; }
LSR_CFG=5 LSR_STEPS=2 timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $OUT/c5_W -o run --output-format csv -- python3 $ROOT/tools/pmc_step.py > $OUT/c5_W.log 2>&1 || { echo W failed; exit 1; }
cd $ROOT
python tools/pmc_issue.py $OUT/c5_sq1 $OUT/c5_sq2 $OUT/cfg5_r04_pmc_issue.json > $OUT/cfg5_r04_pmc_issue.txt
python tools/pmc_traffic.py $OUT/c5_F $OUT/c5_W $OUT/cfg5_r04_pmc_traffic.json > $OUT/cfg5_r04_pmc_traffic.txt
head -6 $OUT/cfg5_r04_pmc_traffic.txt; head -3 $OUT/cfg5_r04_pmc_issue.txt
