#!/bin/bash
# Round-3 probe 19: swar3 vs HEAD (parity subset + interleaved C2 bench + k_map stats), then the
# round-end rehearsal part A of the in-tree HEAD libraries (tools/r03_final.sh).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/p19; mkdir -p $O
step() { echo "== $1 rc=$2"; [ "$2" -eq 0 ] || exit "$2"; }
bash tools/ab.sh "head swar3" 2 > $O/ab.txt 2>&1; rc=$?; cat $O/ab.txt; step "ab bench" $rc
bash tools/ab_kernel.sh "head swar3" "0" "k_map k_reduce" > $O/abk.txt 2>&1; rc=$?; cat $O/abk.txt; step "abk" $rc
PART=a bash tools/r03_final.sh; step "final A" $?
