#!/bin/bash
# Round 4: fused tail launches (k_split_count runs the unit scan in its last
# workgroup, k_unit_uniq_scan the final scan): fast GPU suite, then C2 A/B
# against the previous kernels (build/var_head) interleaved, then k_reduce's
# per-partition phase stamps (tools/r04_x10.sh).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-x11}; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -x -v --timeout 200 --timeout-method thread -m "gpu and not slow" > $O/gpu_fast.log 2>&1; rc=$?
echo "== gpu fast $(tail -1 $O/gpu_fast.log) rc=$rc"; [ $rc -eq 0 ] || exit $rc
bash tools/ab_kernel.sh "head cur head cur" "0" "k_split_count k_unit_scan k_unit_uniq_scan k_final_scan k_reduce k_map" > $O/tail_ab.txt 2>&1; rc=$?
cat $O/tail_ab.txt; [ $rc -eq 0 ] || exit $rc
bash tools/r04_x10.sh ${1:-x11}_st
