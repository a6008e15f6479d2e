#!/bin/bash
# Round-3 probe 1: k_map A/B (direct pass A, one-multiply hash) by kernel
# averages, k_reduce per-partition stamps (ablation build), SQ counters of
# k_map and k_reduce.  Stops at the first failing step.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/p1; mkdir -p $O
step() { echo "== $1 rc=$2"; [ "$2" -eq 0 ] || exit "$2"; }
for v in direct hash1; do
  MOX_LIB=build/var_$v/libmox.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 \
    --timeout-method thread -k "kats or fuzz or tile or corpora or misaligned" > $O/par_$v.log 2>&1
  rc=$?; step "parity $v $(tail -1 $O/par_$v.log)" $rc
done
bash tools/ab_kernel.sh "base direct hash1" "0" "k_map k_reduce" > $O/abk1.txt 2>&1; step "abk round 1" $?
cat $O/abk1.txt
bash tools/ab_kernel.sh "hash1 direct base" "0" "k_map k_reduce" > $O/abk2.txt 2>&1; step "abk round 2" $?
cat $O/abk2.txt
mkdir -p $O/stamps
MOX_LIB=build/var_abl/libmox.so MOX_DBG=1024 MOX_DEBUG_DIR=$O/stamps timeout -k 10 200 python -u bench.py --steps 2 --warmup 1 \
  --no-cpu-baseline > $O/stamps.log 2>&1; step "stamps" $?
python3 tools/stamps.py $O/stamps/stamps.csv > $O/stamps_summary.txt; step "stamps summary" $?
cat $O/stamps_summary.txt
bash tools/pmc_sq.sh k_map p1/sqmap > $O/sqmap.txt 2>&1; step "sq k_map" $?
bash tools/pmc_sq.sh 'k_reduce$' p1/sqred > $O/sqred.txt 2>&1; step "sq k_reduce" $?
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_exchange.py tests/test_gpu_collide.py -x -q --timeout 150 \
  --timeout-method thread > $O/par_main.log 2>&1; rc=$?; step "parity main $(tail -1 $O/par_main.log)" $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c2 -o run -- python3 bench.py --steps 10 --warmup 2 \
  --no-cpu-baseline > $O/c2_under_rocprof.log 2>&1; step "rocprof C2" $?
python3 tools/trace_timeline.py $O/c2 > $O/c2_timeline.txt; step "timeline C2" $?
cat $O/c2_timeline.txt
timeout -k 10 200 build/ingest_probe /tmp/mox_ingest_probe.bin 1024 > $O/ingest_probe.txt 2>&1; step "ingest probe" $?
cat $O/ingest_probe.txt
