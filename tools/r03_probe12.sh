#!/bin/bash
# Round-3 probe 12: the next pass's side dictionary build waits for this pass's k_map (mw)
# vs free-running (head), and workgroup-major cold_n again (rm): C2 end-to-end bench, then the
# evidence-B steps (C4 / C5 bench lines, C4 timeline, N = 2 engine group).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/p12; mkdir -p $O
step() { echo "== $1 rc=$2"; [ "$2" -eq 0 ] || exit "$2"; }
bash tools/ab.sh "head mw rm" 2 > $O/ab.txt 2>&1; step "ab bench" $?
cat $O/ab.txt
bash tools/r03_evidB.sh evB; step "evidence B" $?
