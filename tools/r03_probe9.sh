#!/bin/bash
# Round-3 probe 9: k_reduce takes whole partitions biggest first (lpt) vs the
# double-buffered-dictionary build (dset): parity on the reduce-heavy tests,
# kernel averages, end-to-end bench.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/p9; mkdir -p $O
step() { echo "== $1 rc=$2"; [ "$2" -eq 0 ] || exit "$2"; }
MOX_LIB=build/var_lpt/libmox.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_exchange.py -x -q --timeout 200 \
  --timeout-method thread -k "kats or corpora or split or high or exchange or dictionary or async" > $O/par_lpt.log 2>&1
step "parity lpt $(tail -1 $O/par_lpt.log)" $?
bash tools/ab_kernel.sh "dset lpt" "0" "k_reduce k_unit_scan k_map" > $O/abk1.txt 2>&1; step "abk 1" $?
cat $O/abk1.txt
bash tools/ab_kernel.sh "lpt dset" "0" "k_reduce k_unit_scan k_map" > $O/abk2.txt 2>&1; step "abk 2" $?
cat $O/abk2.txt
bash tools/ab.sh "dset lpt" 2 > $O/ab.txt 2>&1; step "ab bench" $?
cat $O/ab.txt
for cfg in "1 1" "0 1" "1 0" "0 0"; do
  set -- $cfg
  if [ "$2" = "0" ]; then export HSA_ENABLE_SDMA=0; else unset HSA_ENABLE_SDMA; fi
  MOX_FILE_STREAMS=$1 timeout -k 10 200 python -u tools/ingest_bench.py > $O/ing_s$1_sdma$2.txt 2>&1
  step "ingest streams=$1 sdma=$2" $?
  tail -2 $O/ing_s$1_sdma$2.txt | cut -c1-120
done
unset HSA_ENABLE_SDMA
