#!/bin/bash
# Round-3 ingest A/B: mox_count_file end to end on a 1 GiB C2 file in /dev/shm,
# per-reader copy streams (MOX_FILE_STREAMS=0) vs one shared copy stream, 8 / 12 /
# 16 reader threads; then the file-API parity tests.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/ing; mkdir -p $O
step() { echo "== $1 rc=$2"; [ "$2" -eq 0 ] || exit "$2"; }
for cfg in "0 8" "1 8" "1 12" "1 16" "0 16"; do
  set -- $cfg
  MOX_FILE_STREAMS=$1 MOX_FILE_READERS=$2 timeout -k 10 200 python -u tools/ingest_bench.py > $O/ing_$1_$2.txt 2>&1
  step "ingest streams=$1 readers=$2" $?
  tail -2 $O/ing_$1_$2.txt | cut -c1-160
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_group.py -x -q --timeout 200 --timeout-method thread \
  -k "file or cli" > $O/par_file.log 2>&1; rc=$?; step "file parity $(tail -1 $O/par_file.log)" $rc
