#!/bin/bash
# map-kernel ablation (MOX_DBG bits: 1 no tokens, 2 no emit, 4 no dict probe, 8 no cold store, 16 no dict add)
for d in ${DBGS:-0 1 2 4 8 16}; do
  echo "== MOX_DBG=$d"
  MOX_DBG=$d timeout -k 10 120 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/ablate_$d.log 2>&1 || { tail -5 gpurun_out/ablate_$d.log; continue; }
  tail -1 gpurun_out/ablate_$d.log | python -c "
import json,sys; l=json.loads(sys.stdin.readline()); print('GB/s', l['value'], l['phases_ms'])"
done
