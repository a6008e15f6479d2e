#!/bin/bash
# per-kernel time of the bench workload (rocprofv3 kernel-trace stats)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${1:-ks}; shift
OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline "$@" > $OUT/bench.log 2>&1
rc=$?; echo "rc=$rc"; tail -1 $OUT/bench.log | cut -c1-300
cut -d, -f1-4 $OUT/run_kernel_stats.csv
exit $rc
