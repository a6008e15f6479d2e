#!/bin/bash
# Round-3 probe 6: dictionary build with one cuckoo relocation per failed word
# (kick) vs plain 2-choice greedy (new): parity, end-to-end bench, kernel averages.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/p6; mkdir -p $O
step() { echo "== $1 rc=$2"; [ "$2" -eq 0 ] || exit "$2"; }
bash tools/ab.sh "new kick" 2 > $O/ab.txt 2>&1; step "ab bench" $?
cat $O/ab.txt
bash tools/ab_kernel.sh "new kick" "0" "k_map k_reduce k_dict_build" > $O/abk1.txt 2>&1; step "abk" $?
cat $O/abk1.txt
