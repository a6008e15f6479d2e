#!/bin/bash
# Round-3 probe 3: token passes with all LDS reads of a pass issued before use
# (sched barriers) vs the previous build, file ingest through one copy stream
# and the map overlapped with the ingest.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/p3; mkdir -p $O
step() { echo "== $1 rc=$2"; [ "$2" -eq 0 ] || exit "$2"; }
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread \
  -k "file or kats or fuzz or tile or corpora or split or dictionary" > $O/par_main.log 2>&1; rc=$?; step "parity main $(tail -1 $O/par_main.log)" $rc
bash tools/ab_kernel.sh "base fence" "0" "k_map k_reduce" > $O/abk1.txt 2>&1; step "abk round 1" $?
cat $O/abk1.txt
bash tools/ab_kernel.sh "fence base" "0" "k_map k_reduce" > $O/abk2.txt 2>&1; step "abk round 2" $?
cat $O/abk2.txt
bash tools/r03_ingest.sh > $O/ingest.txt 2>&1; step "ingest" $?
cat $O/ingest.txt
