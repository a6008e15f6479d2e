#!/bin/bash
# Round-3 end rehearsal on the final tree.  PART=a: fast GPU suite, smoke(), default bench line,
# rocprofv3 kernel stats + pass timeline of the bench.  PART=b: the slow GPU tests.  Every GPU step
# has its own time limit; the script stops at the first failure.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/final; mkdir -p $O
step() { echo "== $1 rc=$2"; [ "$2" -eq 0 ] || exit "$2"; }
if [ "${PART:-a}" = a ]; then
  timeout -k 10 540 python -u -m pytest tests -m "gpu and not slow" -v --timeout 200 --timeout-method thread > $O/gpu_fast.log 2>&1
  rc=$?; step "gpu fast $(tail -1 $O/gpu_fast.log)" $rc
  timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1
  rc=$?; step "smoke $(tail -1 $O/smoke.log)" $rc
  timeout -k 10 300 python -u bench.py > $O/bench_c2.json 2> $O/bench_c2.err; step "bench C2" $?
  cut -c1-400 $O/bench_c2.json
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c2 -o run -- python3 bench.py --steps 10 --warmup 2 \
    --no-cpu-baseline > $O/c2_under_rocprof.log 2>&1; step "rocprof C2" $?
  python3 tools/trace_timeline.py $O/c2 > $O/c2_timeline.txt; step "timeline C2" $?
  tail -1 $O/c2_timeline.txt
else
  timeout -k 10 600 python -u -m pytest tests -m "gpu and slow" -v --timeout 400 --timeout-method thread > $O/gpu_slow.log 2>&1
  rc=$?; step "gpu slow $(tail -1 $O/gpu_slow.log)" $rc
fi
