#!/bin/bash
# Round-5 (session 3): two-rank rehearsal of bench.py's data-parallel path on the one GPU
# of the box (both ranks on cuda:0, gloo exchange): cfg3 and cfg5.
set -u
OUT=gpurun_out; mkdir -p $OUT
export LSR_BENCH_BACKEND=gloo LSR_BENCH_SAME_DEVICE=1
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --steps 5 --warmup 2 --no-cpu-baseline --no-fwd-1mpix --no-quick > $OUT/r05s3_rehearse2_cfg3.json 2> $OUT/r05s3_rehearse2_cfg3.err || { echo "cfg3 rehearsal failed"; tail -30 $OUT/r05s3_rehearse2_cfg3.err; exit 1; }
cat $OUT/r05s3_rehearse2_cfg3.json
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29532 bench.py --gpus 2 --config 5 --steps 5 --warmup 2 --no-cpu-baseline > $OUT/r05s3_rehearse2_cfg5.json 2> $OUT/r05s3_rehearse2_cfg5.err || { echo "cfg5 rehearsal failed"; tail -30 $OUT/r05s3_rehearse2_cfg5.err; exit 1; }
cat $OUT/r05s3_rehearse2_cfg5.json
echo done
