#!/bin/bash
# GPU: full parity suite (not slow), then per-kernel stats of C2 and a 1 GiB C4.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -k "not slow" > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
bash tools/kstats.sh ks_c2 && bash tools/kstats.sh ks_c4 --workload C4 --bytes-per-gpu ${C4B:-1073741824}
