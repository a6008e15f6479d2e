#!/bin/bash
# GPU: parity tests (incl. the high-cardinality split), then C2 and C4 bench lines.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread -k "not slow" ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -30 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench.log | cut -c1-1500
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --workload C4 ${C4_ARGS} > gpurun_out/c4.log 2>&1
rc=$?; echo "c4 rc=$rc"; tail -1 gpurun_out/c4.log | cut -c1-1800
exit $rc
