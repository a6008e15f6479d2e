#!/bin/bash
# C4 (16 GiB high-cardinality) bench line + kernel trace timeline of one pass.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${1:-c4p}; O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 400 python -u bench.py --workload C4 --steps 3 --warmup 1 --no-cpu-baseline > $O/bench.json 2> $O/bench.err
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/bench.err; exit $rc; }
python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['phases_ms'])" $O/bench.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --workload C4 \
  --steps 2 --warmup 1 --no-cpu-baseline > $O/prof.log 2>&1
rc=$?; echo "rocprof rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 tools/trace_timeline.py $O/prof
