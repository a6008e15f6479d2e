#!/bin/bash
# Round-3 probe 15: k_map consumer reads the slot flag and data in one LDS round trip (spec), and also takes its next ticket ahead (specpf), vs HEAD
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/p15; mkdir -p $O
step() { echo "== $1 rc=$2"; [ "$2" -eq 0 ] || exit "$2"; }
bash tools/ab.sh "head spec specpf" 3 > $O/ab.txt 2>&1; rc=$?; cat $O/ab.txt; step "ab bench" $rc
bash tools/ab_kernel.sh "head spec specpf" "0" "k_map k_reduce" > $O/abk.txt 2>&1; rc=$?; cat $O/abk.txt; step "abk" $rc
