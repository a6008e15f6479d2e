#!/bin/bash
# Round-3 probe 14: key reads of every batch in one LDS round trip (pin), and k_reduce fast path over a chunk at once (joint = pin + MOX_RED_JOINT=1)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/p14; mkdir -p $O
step() { echo "== $1 rc=$2"; [ "$2" -eq 0 ] || exit "$2"; }
bash tools/ab.sh "listv pin joint" 3 > $O/ab.txt 2>&1; rc=$?; cat $O/ab.txt; step "ab bench" $rc
bash tools/ab_kernel.sh "listv pin joint" "0" "k_map k_reduce" > $O/abk.txt 2>&1; rc=$?; cat $O/abk.txt; step "abk" $rc
