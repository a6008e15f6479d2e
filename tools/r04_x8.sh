#!/bin/bash
# Round 4: C4 k_map cold path split (-DMOX_ABLATE build): 8 no cold path,
# 8192 pairs formed but not stored, 16384 every record stored alone (no pair
# slots), 0 full (pairs + stores).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-x8}; mkdir -p $O
bash tools/ab_kernel.sh "abl" "${DBGS:-8 8192 16384 0}" "k_map k_split_count k_split_scatter k_reduce_sort1" --workload C4 --steps 3 --warmup 1 --no-cpu-baseline > $O/c4_cold.txt 2>&1; rc=$?
cat $O/c4_cold.txt; exit $rc
