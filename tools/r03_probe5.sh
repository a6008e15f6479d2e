#!/bin/bash
# Round-3 probe 5: the 2-choice single-slot dictionary with one token pass
# (new) against the committed build (old), plus partition-major cold_n (pm)
# and the LDS-only barrier after k_reduce's write-out (lb) on the old
# dictionary: GPU suite on the new build, kernel averages, end-to-end bench.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/p5; mkdir -p $O
step() { echo "== $1 rc=$2"; [ "$2" -eq 0 ] || exit "$2"; }
timeout -k 10 600 python -u -m pytest tests -m "gpu and not slow" -x -q --timeout 300 --timeout-method thread > $O/gpu_fast.log 2>&1; rc=$?; step "gpu fast $(tail -1 $O/gpu_fast.log)" $rc
bash tools/ab_kernel.sh "old pm lb new" "0" "k_map k_reduce k_hist" > $O/abk1.txt 2>&1; step "abk round 1" $?
cat $O/abk1.txt
bash tools/ab_kernel.sh "new lb pm old" "0" "k_map k_reduce k_hist" > $O/abk2.txt 2>&1; step "abk round 2" $?
cat $O/abk2.txt
bash tools/ab.sh "old new" 2 > $O/ab.txt 2>&1; step "ab bench" $?
cat $O/ab.txt
