#!/bin/bash
# Round-end rehearsal of what the driver runs: GPU suite (SEL=gpu: all, default: fast; SUITE_TIMEOUT seconds),
# smoke(), default bench.py.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-final}; mkdir -p $O
timeout -k 10 ${SUITE_TIMEOUT:-420} python -u -m pytest tests -m "${SEL:-gpu and not slow}" -v --timeout 600 --timeout-method thread > $O/gpu_fast.log 2>&1
rc=$?; echo "fast rc=$rc $(tail -1 $O/gpu_fast.log)"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc $(tail -1 $O/smoke.log)"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.err
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || exit $rc; cut -c1-300 $O/bench.json
