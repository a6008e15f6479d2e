#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -k "split or cardinality or kats" > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
bash tools/kstats.sh ks_c2 && bash tools/kstats.sh ks_c4 --workload C4 --bytes-per-gpu ${C4B:-4294967296}
