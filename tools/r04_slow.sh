#!/bin/bash
# Round 4: the slow GPU tests (full-size C2 / C4 / C5 checks and the C3
# two-shard engine-group test) on this tree.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-slow}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_group.py tests/test_table_sort.py -x -v --timeout 200 --timeout-method thread -m "gpu and not slow" > $O/group_tests.log 2>&1; rc=$?; tail -1 $O/group_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 1000 python -u -m pytest tests -v --timeout 600 --timeout-method thread -m "gpu and slow" > $O/gpu_slow.log 2>&1; rc=$?
tail -15 $O/gpu_slow.log; echo "== slow rc=$rc"; exit $rc
