set -e
ROOT=$(pwd); OUT=$ROOT/gpurun_out/pmcbwd; mkdir -p $OUT; export TMPDIR=/tmp; cd /tmp
P1="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_BRANCH"
P2="SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_INST_CYCLES_VMEM_WR SQ_INSTS_VMEM_WR"
for v in mf legacy; do
  if [ $v = mf ]; then L=$ROOT/langsplatv2_amd/liblsr.so; else L=$ROOT/langsplatv2_amd/_build/var_legacy_exact/liblsr.so; fi
  LSR_LIB=$L LSR_STEPS=2 timeout -k 10 300 rocprofv3 --pmc $P1 -d $OUT/${v}_p1 -o run --output-format csv -- python3 $ROOT/tools/pmc_step.py > $OUT/${v}_p1.log 2>&1
  LSR_LIB=$L LSR_STEPS=2 timeout -k 10 300 rocprofv3 --pmc $P2 -d $OUT/${v}_p2 -o run --output-format csv -- python3 $ROOT/tools/pmc_step.py > $OUT/${v}_p2.log 2>&1
done
cd $ROOT
python tools/pmc_kernel.py $OUT/mf_p1 k_render_bwd $OUT/mf_p2 k_render_bwd $OUT/legacy_p1 k_render_bwd $OUT/legacy_p2 k_render_bwd
