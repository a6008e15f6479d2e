#!/bin/bash
# Round-3 probe 16: token-pass key window read as dwords at the 4-aligned start (keydw) vs HEAD
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/p16; mkdir -p $O
step() { echo "== $1 rc=$2"; [ "$2" -eq 0 ] || exit "$2"; }
bash tools/ab.sh "head keydw" 3 > $O/ab.txt 2>&1; rc=$?; cat $O/ab.txt; step "ab bench" $rc
bash tools/ab_kernel.sh "head keydw" "0" "k_map k_reduce" > $O/abk.txt 2>&1; rc=$?; cat $O/abk.txt; step "abk" $rc
