#!/bin/bash
# Round-3 probe 13: token-list loop with raw v_ffbl and a per-lane base pointer
# (listv) vs HEAD: parity + interleaved C2 bench, then k_map kernel stats.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/p13; mkdir -p $O
step() { echo "== $1 rc=$2"; [ "$2" -eq 0 ] || exit "$2"; }
bash tools/ab.sh "head listv" 3 > $O/ab.txt 2>&1; rc=$?; cat $O/ab.txt; step "ab bench" $rc
bash tools/ab_kernel.sh "head listv" "0" "k_map k_reduce" > $O/abk.txt 2>&1; rc=$?; cat $O/abk.txt; step "abk" $rc
