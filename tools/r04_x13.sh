#!/bin/bash
# fast GPU suite + the 4 GiB C4 digest test on the working tree (k_map rare
# paths settled, k_split_scatter chunk pipeline, k_reduce_sort1 without
# spills), then head (4285063) vs cur interleaved at C2 and C4
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-x13}; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -x -v --timeout 200 --timeout-method thread -m "gpu and not slow" > $O/gpu_fast.log 2>&1; rc=$?
echo "== gpu fast $(tail -1 $O/gpu_fast.log) rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u -m pytest tests/test_gpu_scale.py -x -v --timeout 300 --timeout-method thread -m gpu -k c4_4gib > $O/c4_4gib.log 2>&1; rc=$?
echo "== c4 4gib $(tail -1 $O/c4_4gib.log) rc=$rc"; [ $rc -eq 0 ] || exit $rc
bash tools/ab_kernel.sh "head cur head cur" "0" "k_map k_reduce" > $O/ab_c2.txt 2>&1; rc=$?; cat $O/ab_c2.txt; [ $rc -eq 0 ] || exit $rc
bash tools/ab_kernel.sh "head cur cur head" "0" "k_map k_split_count k_split_scatter k_reduce_sort1 k_mat" --workload C4 --steps 3 --warmup 1 --no-cpu-baseline > $O/ab_c4.txt 2>&1; rc=$?; cat $O/ab_c4.txt; exit $rc
