#!/bin/bash
# Bench lines for every single-GPU config (C2 default with the CPU baseline, C5,
# C4 at 16 GiB) plus the N=2 code path with two ranks sharing GPU 0 over the
# host transport (bench's multi-rank logic; RCCL needs distinct GPUs).
set -o pipefail
mkdir -p gpurun_out
run() { local tag=$1; shift; timeout -k 10 420 python -u bench.py "$@" > gpurun_out/bench_$tag.log 2>&1; local rc=$?; echo "$tag rc=$rc"; tail -1 gpurun_out/bench_$tag.log | cut -c1-400; return $rc; }
run c2 --steps 10 --warmup 3 && \
run c5 --steps 5 --warmup 2 --no-cpu-baseline --workload C5 && \
run c4 --steps 3 --warmup 2 --no-cpu-baseline --workload C4 && \
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 2 --xport host --device 0 --no-cpu-baseline > gpurun_out/bench_n2host.log 2>&1; echo "n2host rc=$?"; tail -1 gpurun_out/bench_n2host.log | cut -c1-400
