#!/bin/bash
# bench.py's N>1 path with ranks sharing the one GPU of a gpurun box:
# host-staged transport, then (experiment) RCCL with two ranks on one device.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29571 \
  bench.py --gpus 2 --steps 5 --warmup 2 --device 0 --xport host --bytes-per-gpu 268435456 > gpurun_out/multi_host.log 2>&1
rc=$?; echo "host rc=$rc"; tail -2 gpurun_out/multi_host.log | cut -c1-1500
[ $rc -eq 0 ] || exit $rc
NCCL_DEBUG=WARN timeout -k 10 120 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29572 \
  bench.py --gpus 2 --steps 5 --warmup 2 --device 0 --xport rccl --bytes-per-gpu 268435456 > gpurun_out/multi_rccl.log 2>&1
rc=$?; echo "rccl rc=$rc"; grep -v "^\s*$" gpurun_out/multi_rccl.log | tail -8 | cut -c1-600
exit $rc
