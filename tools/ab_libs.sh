#!/bin/bash
# A/B of several libmox builds on the bench: LIBS="tag1:path1 tag2:path2 ..." [bench args]
mkdir -p gpurun_out
for spec in $LIBS; do
  tag=${spec%%:*}; lib=${spec#*:}
  MOX_LIB=$lib timeout -k 10 150 python -u bench.py --steps ${STEPS:-10} --warmup 3 --no-cpu-baseline "$@" > gpurun_out/ab_$tag.log 2>&1 || { echo "$tag failed"; tail -5 gpurun_out/ab_$tag.log; exit 1; }
  tail -1 gpurun_out/ab_$tag.log | python -c "
import json,sys; l=json.loads(sys.stdin.readline()); print('$tag GB/s', l['value'], 'ok', l['check_sum_counts_eq_tokens'], l['phases_ms'])"
done
