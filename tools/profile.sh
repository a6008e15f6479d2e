#!/bin/bash
# rocprofv3 evidence for the bench workload: kernel-trace stats, then one PMC
# pass per TCC counter (FETCH_SIZE and WRITE_SIZE cannot share a pass).
# Usage (on the GPU box): bash tools/profile.sh TAG [bench args...]
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${1:-r01}; shift
ARGS=${@:---steps 10 --warmup 2 --no-cpu-baseline}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats -o run -- python3 bench.py $ARGS > $OUT/bench_stats.log 2>&1
rc=$?; echo "stats rc=$rc"; tail -2 $OUT/bench_stats.log; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex k_map --output-format csv -d $OUT/fetch -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > $OUT/bench_fetch.log 2>&1
rc=$?; echo "fetch rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex k_map --output-format csv -d $OUT/write -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > $OUT/bench_write.log 2>&1
rc=$?; echo "write rc=$rc"; [ $rc -eq 0 ] || exit $rc
find $OUT -name "*.csv" | head -20
