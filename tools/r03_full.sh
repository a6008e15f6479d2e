#!/bin/bash
# Round-3 evidence run: GPU suite (fast + slow), C2 bench line + kernel trace +
# timeline, C4 / C5 bench lines, C4 timeline, N = 2 bench through the engine
# group on one GPU.  Every GPU step has its own time limit; stops at the first
# failure.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${1:-full}; O=gpurun_out/$TAG; mkdir -p $O
step() { echo "== $1 rc=$2"; [ "$2" -eq 0 ] || exit "$2"; }
timeout -k 10 600 python -u -m pytest tests -m "gpu and not slow" -v --timeout 300 --timeout-method thread > $O/gpu_fast.log 2>&1; rc=$?; step "gpu fast $(tail -1 $O/gpu_fast.log)" $rc
timeout -k 10 700 python -u -m pytest tests -m "gpu and slow" -v --timeout 600 --timeout-method thread > $O/gpu_slow.log 2>&1; rc=$?; step "gpu slow $(tail -1 $O/gpu_slow.log)" $rc
timeout -k 10 300 python -u bench.py > $O/bench_c2.json 2> $O/bench_c2.err; step "bench C2" $?
cut -c1-200 $O/bench_c2.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c2 -o run -- python3 bench.py --steps 10 --warmup 2 \
  --no-cpu-baseline > $O/c2_under_rocprof.log 2>&1; step "rocprof C2" $?
python3 tools/trace_timeline.py $O/c2 > $O/c2_timeline.txt; step "timeline C2" $?
tail -1 $O/c2_timeline.txt
timeout -k 10 420 python -u bench.py --workload C4 --steps 5 --warmup 2 --cpu-sample-mib 256 > $O/bench_c4.json 2> $O/bench_c4.err; step "bench C4" $?
cut -c1-200 $O/bench_c4.json
timeout -k 10 420 python -u bench.py --workload C5 --steps 5 --warmup 2 --cpu-sample-mib 1024 > $O/bench_c5.json 2> $O/bench_c5.err; step "bench C5" $?
cut -c1-200 $O/bench_c5.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c4 -o run -- python3 bench.py --workload C4 \
  --steps 2 --warmup 1 --no-cpu-baseline > $O/c4_under_rocprof.log 2>&1; step "rocprof C4" $?
python3 tools/trace_timeline.py $O/c4 > $O/c4_timeline.txt; step "timeline C4" $?
tail -1 $O/c4_timeline.txt
timeout -k 10 300 python -u bench.py --gpus 2 --xport host --device 0 --steps 5 --warmup 2 --no-cpu-baseline > $O/bench_n2_group.json 2> $O/bench_n2_group.err; step "bench N=2 group" $?
cut -c1-300 $O/bench_n2_group.json
