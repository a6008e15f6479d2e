#!/bin/bash
# High-cardinality path: parity tests of the split / small-unit reduce, then the
# C4 bench line and its kernel stats.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/c4; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_exchange.py tests/test_gpu_scale.py -x -q \
  --timeout 400 --timeout-method thread -k "${TESTS:-split or cardinality or bounds or c4_4gib or async}" > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc $(tail -1 $O/tests.log)"; [ $rc -eq 0 ] || { tail -30 $O/tests.log; exit $rc; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --workload C4 \
  --steps 4 --warmup 2 --no-cpu-baseline > $O/bench.json 2> $O/bench.err
rc=$?; echo "bench C4 rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/bench.err; exit $rc; }
python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('C4 GB/s', d['value'], 'ms', d['ms_per_step'], d['phases_ms'])" $O/bench.json
cut -d, -f1-4 $O/prof/run_kernel_stats.csv | head -12
