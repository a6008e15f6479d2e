#!/bin/bash
# Round 4 evidence A: the fast GPU suite, the default bench line (C2 with
# the CPU baseline), and a rocprofv3 kernel trace + stats of the C2 bench with
# one pass's timeline (tools/trace_timeline.py).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-evA}; mkdir -p $O
step() { echo "== $1 rc=$2"; [ "$2" -eq 0 ] || exit "$2"; }
timeout -k 10 700 python -u -m pytest tests -x -v --timeout 200 --timeout-method thread -m "gpu and not slow" > $O/gpu_fast.log 2>&1; rc=$?; step "gpu fast $(tail -1 $O/gpu_fast.log)" $rc
timeout -k 10 400 python -u bench.py > $O/bench_c2.json 2> $O/bench_c2.err; step "bench C2" $?
cut -c1-300 $O/bench_c2.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c2 -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/c2_under_rocprof.log 2>&1; step "rocprof C2" $?
python3 tools/trace_timeline.py $O/c2 > $O/c2_timeline.txt; step "timeline C2" $?
tail -1 $O/c2_timeline.txt
