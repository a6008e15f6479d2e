#!/bin/bash
# Round-3 probe 4: ingest variants (tools/ingest_probe.cpp E/E2/F/G), k_reduce
# batched fast path (rbatch) vs the current build (fence), parity of rbatch.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/p4; mkdir -p $O
step() { echo "== $1 rc=$2"; [ "$2" -eq 0 ] || exit "$2"; }
timeout -k 10 400 build/ingest_probe /tmp/mox_ingest_probe.bin 1024 > $O/ingest_probe.txt 2>&1; step "ingest probe" $?
cat $O/ingest_probe.txt
MOX_LIB=build/var_rbatch/libmox.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_exchange.py -x -q --timeout 200 \
  --timeout-method thread -k "kats or fuzz or corpora or split or high or exchange or dictionary" > $O/par_rbatch.log 2>&1
step "parity rbatch $(tail -1 $O/par_rbatch.log)" $?
bash tools/ab_kernel.sh "fence rbatch" "0" "k_reduce k_map" > $O/abk1.txt 2>&1; step "abk round 1" $?
cat $O/abk1.txt
bash tools/ab_kernel.sh "rbatch fence" "0" "k_reduce k_map" > $O/abk2.txt 2>&1; step "abk round 2" $?
cat $O/abk2.txt
