#!/bin/bash
# Round-3 state check on a GPU box: fast GPU suite (incl. collision build,
# engine group, golden corpora), default C2 bench line, C2 kernel trace +
# pass timeline.  Every GPU step has its own time limit; the script stops
# at the first failure.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${1:-st}; O=gpurun_out/$TAG; mkdir -p $O
step() { echo "== $1 rc=$2"; [ "$2" -eq 0 ] || exit "$2"; }
timeout -k 10 600 python -u -m pytest tests -m "gpu and not slow" -v --timeout 150 --timeout-method thread > $O/gpu_fast.log 2>&1; rc=$?; step "gpu fast $(tail -1 $O/gpu_fast.log)" $rc
timeout -k 10 300 python -u bench.py > $O/bench_c2.json 2> $O/bench_c2.err; step "bench C2" $?
cut -c1-200 $O/bench_c2.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c2 -o run -- python3 bench.py --steps 10 --warmup 2 \
  --no-cpu-baseline > $O/c2_under_rocprof.log 2>&1; step "rocprof C2" $?
python3 tools/trace_timeline.py $O/c2 > $O/c2_timeline.txt; step "timeline C2" $?
tail -1 $O/c2_timeline.txt
