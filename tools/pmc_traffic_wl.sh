#!/bin/bash
# k_map HBM traffic (FETCH / WRITE in separate PMC passes) for one workload:
# profiles-ready summary gpurun_out/TAG/pmc_k_map_WORKLOAD.json.
# Usage: bash tools/pmc_traffic_wl.sh WORKLOAD BYTES_PER_GPU TAG
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
WL=$1; BYTES=$2; O=gpurun_out/${3:-pmcw}_$WL; mkdir -p $O
for c in FETCH_SIZE WRITE_SIZE; do
  d=$( [ $c = FETCH_SIZE ] && echo fetch || echo write )
  timeout -s KILL 240 rocprofv3 --pmc $c --kernel-include-regex k_map --output-format csv -d $O/$d -o run -- python3 bench.py \
    --workload $WL --steps 2 --warmup 1 --no-cpu-baseline > $O/$d.log 2>&1
  rc=$?; echo "$WL $c rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
python3 tools/pmc_traffic.py $O k_map $O/pmc_k_map_$WL.json $WL $BYTES
