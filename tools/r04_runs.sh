#!/bin/bash
# Round-4 GPU runs, one section per call; every file under profiles/r04/ names
# the section that produced it.  Usage on a GPU box (through gpurun):
#   bash tools/r04_runs.sh SECTION [TAG]      (outputs under gpurun_out/TAG)
#
# Sections:
#   evid     fast GPU suite, default C2 bench line (with the CPU baseline), a
#            rocprofv3 kernel trace + stats of the C2 bench and one pass's timeline
#   slow     engine-group / sort GPU tests, then the slow GPU tests (full-size C2,
#            C4, C5 and the C3 two-shard engine-group test)
#   n2       N = 2 engine group bench (2 x 8 GiB C3 shards, device-copy transport,
#            both members on GPU 0) and a kernel + copy + HIP API trace of it
#            (tools/step_timeline.py: the exchange pass)
#   ladder   k_map time ladder at C2 (-DMOX_ABLATE build var_abl, MOX_DBG stages:
#            4096 loader + ring only, 1 + byte phase, 2 + token list, 24 + token
#            pass without dictionary adds and cold stores, 8 + dictionary adds, 0 full)
#   c4abl    C4 k_map stages (4096, 2, 8, 0 as above) and the no-dictionary cold
#            path split (8192 pairs formed but not stored, 16384 records stored
#            alone, 32768 pairs stored at consecutive addresses, 0 pairs stored)
#   redabl   C2 k_reduce ablations (64 no inserts, 128 no slow path, 512 plain
#            count add, 32 no sort, 0 full) and per-partition phase stamps
#            (DBG_STAMP 1024, 1088 = stamps without inserts; tools/stamps.py)
#   ab       interleaved per-kernel A/B of build variants: AB_VARS="v1 v2 v1 v2"
#            AB_KERNELS="k_map k_reduce" [AB_ARGS="--workload C4 ..."]
#            (tools/ab_kernel.sh; variants from tools/build_variant.sh)
#   pmc      k_map FETCH/WRITE traffic at C2 (tools/pmc_traffic_wl.sh) and SQ
#            counters of k_map and k_reduce (tools/pmc_sq.sh)
#   lines    C4 and C5 bench lines, a C4 kernel trace + one pass's timeline
#   c4pmc    C4 FETCH_SIZE / WRITE_SIZE per kernel: k_map and the post-map kernels
#   csort    a k_reduce_sort1 variant (AB_VAR, default cs = -DMOX_S1_CSORT=1 in the
#            commit that had it) against the default build: tables identical
#            (tools/cmp_order.py), parity tests with it, C4 per-kernel A/B, and the
#            sort-twice ablation (DBG_S1_SORT2, builds abl / csabl)
#
# Variants used by the round-4 A/Bs (tools/build_variant.sh NAME FLAGS; SRC= an
# exported older commit for the "head"/"base" arms): ldr -DMOX_LD_BATCH=0,
# noldf -DMOX_LD_FENCE=0, rstat -DMOX_RED_DYN=0, rhome -DMOX_RED_HOME=1,
# os8 -DMOX_OS_ITEMS=8, qfpair -DMOX_SPLIT_STAGE=0, s1w3 -DMOX_S1_WG=3,
# rtab0 -DMOX_RED_TAB=0, abl -DMOX_ABLATE.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
SEC=$1
O=gpurun_out/${2:-$SEC}; mkdir -p $O
step() { echo "== $1 rc=$2"; [ "$2" -eq 0 ] || exit "$2"; }
fast_suite() {
  timeout -k 10 700 python -u -m pytest tests -x -v --timeout 200 --timeout-method thread -m "gpu and not slow" > $O/gpu_fast.log 2>&1
  local rc=$?; step "gpu fast $(tail -1 $O/gpu_fast.log)" $rc
}
case $SEC in
evid)
  fast_suite
  timeout -k 10 400 python -u bench.py > $O/bench_c2.json 2> $O/bench_c2.err; step "bench C2" $?
  cut -c1-200 $O/bench_c2.json
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c2 -o run -- \
    python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/c2_under_rocprof.log 2>&1; step "rocprof C2" $?
  python3 tools/trace_timeline.py $O/c2 > $O/c2_timeline.txt; step "timeline C2" $?
  tail -1 $O/c2_timeline.txt
  ;;
slow)
  timeout -k 10 300 python -u -m pytest tests/test_gpu_group.py tests/test_table_sort.py -x -v --timeout 200 \
    --timeout-method thread -m "gpu and not slow" > $O/group_tests.log 2>&1; step "group tests $(tail -1 $O/group_tests.log)" $?
  timeout -k 10 1000 python -u -m pytest tests -v --timeout 600 --timeout-method thread -m "gpu and slow" > $O/gpu_slow.log 2>&1
  rc=$?; tail -15 $O/gpu_slow.log; step slow $rc
  ;;
n2)
  timeout -k 10 400 python -u bench.py --gpus 2 --xport host --device 0 --steps 3 --warmup 1 > $O/n2.json 2> $O/n2.err; step "bench n2" $?
  python3 -c "import json;d=json.load(open('$O/n2.json'));print(d['value'],d['phases_ms'],d.get('hash_order'))"
  timeout -k 10 500 rocprofv3 --kernel-trace --memory-copy-trace --hip-runtime-trace --output-format csv -d $O/n2t -o run -- \
    python3 bench.py --gpus 2 --xport host --device 0 --steps 2 --warmup 1 > $O/n2t.json 2> $O/n2t.err; step "rocprof n2" $?
  python3 tools/step_timeline.py $O/n2t 100 > $O/n2_timeline.txt; step "timeline" $?
  tail -3 $O/n2_timeline.txt
  ;;
ladder)
  bash tools/ab_kernel.sh "abl" "4096 1 2 24 8 0" "k_map" --steps 10 --warmup 2 --no-cpu-baseline > $O/ladder.txt 2>&1
  rc=$?; cat $O/ladder.txt; step ladder $rc
  ;;
c4abl)
  bash tools/ab_kernel.sh "abl" "4096 2 8 8192 16384 32768 0" "k_map" --workload C4 --steps 3 --warmup 1 --no-cpu-baseline \
    > $O/c4_abl.txt 2>&1; rc=$?; cat $O/c4_abl.txt; step c4abl $rc
  ;;
redabl)
  bash tools/ab_kernel.sh "abl" "0 64 128 512 32" "k_reduce" > $O/red_abl.txt 2>&1; rc=$?; cat $O/red_abl.txt; step redabl $rc
  for d in 1024 1088; do
    mkdir -p $O/s$d
    MOX_LIB=build/var_abl/libmox.so MOX_DBG=$d MOX_DEBUG_DIR=$O/s$d timeout -k 10 200 python -u bench.py --steps 3 --warmup 1 \
      --no-cpu-baseline > $O/s$d.log 2>&1; step "stamps $d" $?
    echo "dbg $d"; python3 tools/stamps.py $O/s$d/stamps.csv
  done
  ;;
ab)
  bash tools/ab_kernel.sh "$AB_VARS" "0" "$AB_KERNELS" ${AB_ARGS:-} > $O/ab.txt 2>&1; rc=$?; cat $O/ab.txt; step ab $rc
  ;;
pmc)
  bash tools/pmc_traffic_wl.sh C2 1073741824 ${2:-pmc}_traffic > $O/traffic.txt 2>&1; rc=$?; tail -5 $O/traffic.txt; step traffic $rc
  bash tools/pmc_sq.sh k_map ${2:-pmc}_sqmap > $O/sq_k_map.txt 2>&1; rc=$?; cat $O/sq_k_map.txt; step "sq k_map" $rc
  bash tools/pmc_sq.sh 'k_reduce$' ${2:-pmc}_sqred > $O/sq_k_reduce.txt 2>&1; rc=$?; cat $O/sq_k_reduce.txt; step "sq k_reduce" $rc
  ;;
lines)
  # C4 / C5 bench lines (production build) and a C4 kernel trace + timeline
  for wl in C4 C5; do
    timeout -k 10 500 python -u bench.py --workload $wl --steps 5 --warmup 2 > $O/bench_$wl.json 2> $O/bench_$wl.err; step "bench $wl" $?
    python3 -c "import json;d=json.loads(open('$O/bench_$wl.json').read().strip().splitlines()[-1]);print('$wl',d['value'],d['ms_per_step'],d['phases_ms'])"
  done
  timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c4 -o run -- \
    python3 bench.py --workload C4 --steps 3 --warmup 1 --no-cpu-baseline > $O/c4_under_rocprof.log 2>&1; step "rocprof C4" $?
  python3 tools/trace_timeline.py $O/c4 > $O/c4_timeline.txt; step "timeline C4" $?
  tail -1 $O/c4_timeline.txt
  ;;
c4pmc)
  # C4 per-kernel HBM traffic (FETCH_SIZE, WRITE_SIZE passes) of k_map and the post-map kernels
  BENCH_ARGS="--workload C4" PMC_GROUPS="FETCH_SIZE WRITE_SIZE,GRBM_GUI_ACTIVE" \
    bash tools/pmc_kernels.sh 'k_map|k_split_count|k_split_scatter|k_reduce_sort1|k_reduce_sort2|k_mat' ${2:-c4pmc}_k \
    > $O/pmc.txt 2>&1; rc=$?; cat $O/pmc.txt; step "c4 pmc" $rc
  ;;
csort)
  V=${AB_VAR:-cs}
  timeout -k 10 300 python3 -u tools/cmp_order.py build/var_$V/libmox.so > $O/cmp_order.txt 2>&1; rc=$?; cat $O/cmp_order.txt; step "cmp order" $rc
  MOX_LIB=build/var_$V/libmox.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 200 \
    --timeout-method thread -m "gpu and not slow" -k "split or high_card or corpora or deterministic or fuzz or kats" > $O/par.log 2>&1
  step "parity $(tail -1 $O/par.log)" $?
  bash tools/ab_kernel.sh "def $V def $V" "0" "k_reduce_sort1 k_reduce_sort2" --workload C4 --steps 3 --warmup 1 --no-cpu-baseline \
    > $O/ab.txt 2>&1; rc=$?; cat $O/ab.txt; step ab $rc
  bash tools/ab_kernel.sh "abl ${V}abl" "0 65536" "k_reduce_sort1" --workload C4 --steps 3 --warmup 1 --no-cpu-baseline \
    > $O/abl.txt 2>&1; rc=$?; cat $O/abl.txt; step abl $rc
  ;;
*)
  echo "unknown section $SEC"; exit 2
  ;;
esac
