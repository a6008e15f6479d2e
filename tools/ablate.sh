#!/bin/bash
# map-kernel ablation (MOX_DBG bits: 1 no tokens, 2 no emit, 4 no dict probe, 8 no cold store, 16 no dict add)
for d in ${DBGS:-0 1 2 4 8 16}; do
  echo "== MOX_DBG=$d"
  MOX_DBG=$d timeout -k 10 120 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline | python -c "
import json,sys; l=json.loads(sys.stdin.readline()); print('GB/s', l['value'], l['phases_ms'], l['stats'])" || exit 1
done
