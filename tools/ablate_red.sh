#!/bin/bash
# reduce-kernel ablation with the -DMOX_ABLATE build (build/abl/libmox.so):
# 32 no sort, 64 no insert, 128 no slow path, 512 plain (non-atomic) add
mkdir -p gpurun_out
for d in ${DBGS:-0 32 64 128 512}; do
  MOX_LIB=${LIB:-build/var_abl/libmox.so} MOX_DBG=$d timeout -k 10 120 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline "$@" > gpurun_out/ablr_$d.log 2>&1 || { echo "dbg $d failed"; tail -5 gpurun_out/ablr_$d.log; exit 1; }
  tail -1 gpurun_out/ablr_$d.log | python -c "
import json,sys; l=json.loads(sys.stdin.readline()); print('dbg $d GB/s', l['value'], l['phases_ms'])"
done
