#!/bin/bash
# dictionary sample-size sweep on the C2 bench (engine default 192 pieces)
mkdir -p gpurun_out
for sp in ${SPS:-192 256 128 320 192 256}; do
  timeout -k 10 120 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --sample-pieces $sp > gpurun_out/sw_$sp.log 2>&1 || { echo "sp=$sp failed"; tail -5 gpurun_out/sw_$sp.log; exit 1; }
  tail -1 gpurun_out/sw_$sp.log | python -c "
import json,sys; l=json.loads(sys.stdin.readline()); print('sp=$sp GB/s', l['value'], 'dict', l['phases_ms']['ms_dict'], 'map', l['roofline']['avg_launch_ms'], 'cold', l['stats']['cold_records'], 'words', l['stats']['dict_words'])"
done
