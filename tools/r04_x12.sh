#!/bin/bash
# fast GPU suite on the working tree, then prev (98173bf) / fuse (fused tail
# launches) / cur (+ k_reduce walk without vmcnt(0)) interleaved at C2
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-x12}; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -x -v --timeout 200 --timeout-method thread -m "gpu and not slow" > $O/gpu_fast.log 2>&1; rc=$?
echo "== gpu fast $(tail -1 $O/gpu_fast.log) rc=$rc"; [ $rc -eq 0 ] || exit $rc
bash tools/ab_kernel.sh "prev fuse cur prev fuse cur" "0" "k_split_count k_unit_scan k_unit_uniq_scan k_final_scan k_reduce k_map" > $O/ab.txt 2>&1; rc=$?
cat $O/ab.txt; exit $rc
