#!/bin/bash
# Round-3 probe 20: slow GPU tests on the final tree (tools/r03_final.sh PART=b), then k_map SQ
# counters of the final kernels (tools/pmc_sq.sh).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/p20; mkdir -p $O
step() { echo "== $1 rc=$2"; [ "$2" -eq 0 ] || exit "$2"; }
PART=b bash tools/r03_final.sh; step "final B" $?
bash tools/pmc_sq.sh k_map p20/sqmap > $O/sqmap.txt 2>&1; rc=$?; cat $O/sqmap.txt; step "sq k_map" $rc
