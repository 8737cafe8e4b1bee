#!/bin/bash
# round 2: counter list + partitioned parity (conditioned + free) at C2 and C5
mkdir -p gpurun_out/r2
export TMPDIR=/tmp
timeout -k 10 60 rocprofv3 -L > gpurun_out/r2/counters.txt 2>&1 || true
timeout -k 10 300 python -u -m torch.distributed.run --nnodes 1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 \
  tools/partition_check.py --config C2 --out gpurun_out/r2/partition_c2_r2.json > gpurun_out/r2/partition_c2.log 2>&1
echo "c2 rc=$?"
timeout -k 10 600 python -u -m torch.distributed.run --nnodes 1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29612 \
  tools/partition_check.py --config C5 --out gpurun_out/r2/partition_c5_r2.json > gpurun_out/r2/partition_c5.log 2>&1
echo "c5 rc=$?"
