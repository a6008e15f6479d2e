#!/bin/bash
# Round-3 evidence A: GPU suite (fast + slow), default C2 bench line (CPU
# baseline), C2 kernel trace + pass timeline, k_map FETCH / WRITE traffic.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${1:-evA}; O=gpurun_out/$TAG; mkdir -p $O
step() { echo "== $1 rc=$2"; [ "$2" -eq 0 ] || exit "$2"; }
timeout -k 10 500 python -u -m pytest tests -m "gpu and not slow" -v --timeout 300 --timeout-method thread > $O/gpu_fast.log 2>&1; rc=$?; step "gpu fast $(tail -1 $O/gpu_fast.log)" $rc
timeout -k 10 500 python -u -m pytest tests -m "gpu and slow" -v --timeout 450 --timeout-method thread > $O/gpu_slow.log 2>&1; rc=$?; step "gpu slow $(tail -1 $O/gpu_slow.log)" $rc
timeout -k 10 200 python -u bench.py > $O/bench_c2.json 2> $O/bench_c2.err; step "bench C2" $?
cut -c1-200 $O/bench_c2.json
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c2 -o run -- python3 bench.py --steps 10 --warmup 2 \
  --no-cpu-baseline > $O/c2_under_rocprof.log 2>&1; step "rocprof C2" $?
python3 tools/trace_timeline.py $O/c2 > $O/c2_timeline.txt; step "timeline C2" $?
tail -1 $O/c2_timeline.txt
bash tools/pmc_traffic_wl.sh C2 1073741824 $TAG/pmc > $O/pmc.log 2>&1; step "pmc C2" $?
cat $O/pmc_C2/pmc_k_map_C2.json 2>/dev/null || ls -R $O | head
