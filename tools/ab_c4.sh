#!/bin/bash
# C4 (16 GiB high-cardinality) A/B: LIBS="tag:path ..." ; bench steps under each library
mkdir -p gpurun_out
for spec in $LIBS; do
  tag=${spec%%:*}; lib=${spec#*:}
  MOX_LIB=$lib timeout -k 10 240 python -u bench.py --workload C4 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/c4_$tag.log 2>&1 || { echo "$tag failed"; tail -5 gpurun_out/c4_$tag.log; exit 1; }
  tail -1 gpurun_out/c4_$tag.log | python -c "
import json,sys; l=json.loads(sys.stdin.readline()); print('$tag GB/s', l['value'], 'ms', l['ms_per_step'], 'ok', l['check_sum_counts_eq_tokens'], l['phases_ms'], l['stats']['uniques'])"
done
