#!/bin/bash
# State check at session start: fast GPU suite, C2 bench line, C4 bench under a kernel trace.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-state}; mkdir -p $O
timeout -k 10 420 python -u -m pytest tests -m "gpu and not slow" -v --timeout 150 --timeout-method thread > $O/gpu_fast.log 2>&1
rc=$?; echo "fast rc=$rc $(tail -1 $O/gpu_fast.log)"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/bench_c2.json 2> $O/bench_c2.err
rc=$?; echo "C2 rc=$rc"; [ $rc -eq 0 ] || exit $rc; cut -c1-200 $O/bench_c2.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c4 -o run -- python3 bench.py --workload C4 \
  --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_c4.json 2> $O/bench_c4.err
rc=$?; echo "C4 rc=$rc"; [ $rc -eq 0 ] || exit $rc; cut -c1-200 $O/bench_c4.json
python3 tools/trace_timeline.py $O/c4 > $O/c4_timeline.txt; cat $O/c4_timeline.txt
