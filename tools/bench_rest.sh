#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 420 python -u bench.py --steps 3 --warmup 2 --no-cpu-baseline --workload C4 > gpurun_out/bench_c4.log 2>&1; rc=$?; echo "c4 rc=$rc"; tail -1 gpurun_out/bench_c4.log | cut -c1-1600
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 2 --xport host --device 0 --no-cpu-baseline > gpurun_out/bench_n2host.log 2>&1; echo "n2host rc=$?"; tail -3 gpurun_out/bench_n2host.log | cut -c1-600
