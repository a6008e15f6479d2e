#!/bin/bash
# Round-3 probe 10: GPU suite on the current build (double-buffered dictionary,
# k_reduce biggest partitions first), end-to-end A/B kick -> dset -> lpt,
# k_reduce / k_unit_scan averages, per-row k_map phase cycles, k_map SQ counters.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/p10; mkdir -p $O/st
step() { echo "== $1 rc=$2"; [ "$2" -eq 0 ] || exit "$2"; }
timeout -k 10 600 python -u -m pytest tests -m "gpu and not slow" -x -q --timeout 300 --timeout-method thread > $O/gpu_fast.log 2>&1; rc=$?; step "gpu fast $(tail -1 $O/gpu_fast.log)" $rc
bash tools/ab.sh "kick lpt cbatch" 2 > $O/ab.txt 2>&1; step "ab bench" $?
cat $O/ab.txt
bash tools/ab_kernel.sh "dset lpt cbatch" "0" "k_reduce k_unit_scan k_map" > $O/abk1.txt 2>&1; step "abk 1" $?
cat $O/abk1.txt
MOX_LIB=build/var_stamp/libmox.so MOX_DBG=1024 MOX_DEBUG_DIR=$O/st timeout -k 10 200 python -u bench.py --steps 2 --warmup 1 \
  --no-cpu-baseline > $O/stamp.log 2>&1; step "stamp bench" $?
python3 tools/mapcyc.py $O/st/mapcyc.csv; step "mapcyc" $?
bash tools/pmc_sq.sh k_map p10/sqmap > $O/sqmap.txt 2>&1; step "sq k_map" $?
cat $O/sqmap.txt
