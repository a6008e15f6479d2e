#!/bin/bash
# Round-5 GPU runs, one section per call; every file under profiles/r05/ names
# the section that produced it.  Usage on a GPU box (through gpurun):
#   bash tools/r05_runs.sh SECTION [TAG]      (outputs under gpurun_out/TAG)
#
# Sections:
#   newtests the round-5 tests: full-size async bench-mode C2 parity, the
#            8-member engine group, bench.py --gpus 8 (engine group) and the
#            torchrun launch shape on one GPU, the device sort tests
#   evid     default C2 bench line (with the CPU baseline) and a rocprofv3
#            kernel trace + stats of the C2 bench with one pass's timeline
#   fast     the fast GPU suite (gpu and not slow)
#   parity   the parity subset (test_gpu_parity, test_gpu_collide; not slow)
#   slow     the slow GPU tests
#   ab       interleaved per-kernel A/B of build variants: AB_VARS="v1 v2 v1 v2"
#            AB_KERNELS="k_map" [AB_DBG="0"] [AB_ARGS="--workload C4 ..."]
#   lines    bench lines of C5, C4 and the N = 2 engine group (C3 shards on GPU 0)
#   pmc      k_map FETCH/WRITE traffic at C2 and SQ counters of k_map
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
SEC=$1
O=gpurun_out/${2:-$SEC}; mkdir -p $O
step() { echo "== $1 rc=$2"; [ "$2" -eq 0 ] || exit "$2"; }
pyt() {  # pyt LOG TIMEOUT pytest-args...
  local log=$1 to=$2; shift 2
  timeout -k 10 $to python -u -m pytest -x -v --timeout 600 --timeout-method thread "$@" > $O/$log 2>&1
  local rc=$?; step "$log $(tail -1 $O/$log)" $rc
}
case $SEC in
newtests)
  pyt sort.log 300 tests/test_table_sort.py tests/test_gpu_group.py -m gpu -k "sort"
  pyt group8.log 600 tests/test_gpu_group.py -m gpu -k "eight or torchrun"
  pyt async_c2.log 400 tests/test_gpu_scale.py -m gpu -k "async_bench_mode"
  ;;
evid)
  timeout -k 10 400 python -u bench.py > $O/bench_c2.json 2> $O/bench_c2.err; step "bench C2" $?
  cut -c1-300 $O/bench_c2.json
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c2 -o run -- \
    python3 bench.py --no-cpu-baseline > $O/c2_under_rocprof.log 2>&1; step "rocprof C2" $?
  python3 tools/trace_timeline.py $O/c2 > $O/c2_timeline.txt; step "timeline C2" $?
  tail -1 $O/c2_timeline.txt
  ;;
fast)
  pyt gpu_fast.log 900 tests -m "gpu and not slow"
  ;;
parity)
  # the parity subset of the GPU suite (every k_map path: KATs with and without
  # the dictionary, fuzz, tile edges, corpora, huge tokens, misaligned ranges,
  # split partitions, async passes, file ingest, forced collisions)
  pyt parity.log 700 tests/test_gpu_parity.py tests/test_gpu_collide.py tests/test_gpu_exchange.py -m "gpu and not slow"
  ;;
slow)
  pyt gpu_slow.log 1100 tests -m "gpu and slow"
  ;;
ab)
  bash tools/ab_kernel.sh "$AB_VARS" "${AB_DBG:-0}" "$AB_KERNELS" ${AB_ARGS:-} > $O/ab.txt 2>&1; rc=$?; cat $O/ab.txt; step ab $rc
  ;;
mapdiag)
  # k_map row supply A/B (build variants of tools/build_variant.sh): per-row
  # consumer cycles (-DMOX_STAMP builds, MOX_DBG=1024) and the supply floor
  # (-DMOX_ABLATE builds, MOX_DBG=4096: rows released untouched)
  for v in ${DIAG_STAMP:-ringst selfst}; do
    mkdir -p $O/$v
    MOX_LIB=build/var_$v/libmox.so MOX_DBG=1024 MOX_DEBUG_DIR=$O/$v timeout -k 10 200 python -u bench.py --steps 3 --warmup 1 \
      --no-cpu-baseline > $O/$v.log 2>&1; step "stamps $v" $?
    echo "$v"; python3 tools/mapcyc.py $O/$v/mapcyc.csv
  done
  bash tools/ab_kernel.sh "${DIAG_ABL:-ringabl selfabl}" "4096 0" "k_map" > $O/floor.txt 2>&1; rc=$?; cat $O/floor.txt; step floor $rc
  ;;
xsort)
  # the sorted exchange: exchange + group tests, the C3 2 x 8 GiB group test,
  # and the N = 2 engine-group bench line (2 x 8 GiB C3 shards on GPU 0)
  pyt xsort_tests.log 900 tests/test_gpu_exchange.py tests/test_gpu_group.py -m "gpu and not slow"
  pyt xsort_c3.log 900 tests/test_gpu_scale.py -m gpu -k "c3_group"
  timeout -k 10 400 python -u bench.py --gpus 2 --xport host --device 0 --steps 3 --warmup 1 > $O/n2.json 2> $O/n2.err; step "bench n2" $?
  python3 -c "import json;d=json.load(open('$O/n2.json'));print(d['value'],d['phases_ms'],d.get('hash_order'))"
  ;;
varc2)
  # a build variant's C2 table against the oracle (full size, the bench's async mode)
  MOX_LIB=build/var_${VAR}/libmox.so pyt varc2_$VAR.log 400 tests/test_gpu_scale.py -m gpu -k "async_bench_mode"
  ;;
stages)
  # k_map SQ instruction counts per ablation stage (tools/pmc_map_stages.sh, build/var_abl)
  bash tools/pmc_map_stages.sh ${2:-stages} "${STAGES:-4096 1 2 8 16 0}" > $O/stages.txt 2>&1; rc=$?; cat $O/stages.txt; step stages $rc
  ;;
lines)
  # bench lines of the other configs: C5, C4 (16 GiB each), and the N = 2
  # engine group (2 x 8 GiB C3 shards on GPU 0, device-copy transport, sorted result)
  timeout -k 10 420 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --workload C5 > $O/bench_c5.json 2> $O/bench_c5.err; step "bench C5" $?
  cut -c1-200 $O/bench_c5.json
  timeout -k 10 600 python -u bench.py --steps 3 --warmup 2 --no-cpu-baseline --workload C4 > $O/bench_c4.json 2> $O/bench_c4.err; step "bench C4" $?
  cut -c1-200 $O/bench_c4.json
  timeout -k 10 500 python -u bench.py --gpus 2 --xport host --device 0 --steps 3 --warmup 1 > $O/bench_n2.json 2> $O/bench_n2.err; step "bench N2 group" $?
  cut -c1-200 $O/bench_n2.json
  ;;
pmc)
  bash tools/pmc_traffic_wl.sh C2 1073741824 ${2:-pmc}_traffic > $O/traffic.txt 2>&1; rc=$?; tail -5 $O/traffic.txt; step traffic $rc
  bash tools/pmc_sq.sh k_map ${2:-pmc}_sqmap > $O/sq_k_map.txt 2>&1; rc=$?; cat $O/sq_k_map.txt; step "sq k_map" $rc
  ;;
*)
  echo "unknown section $SEC"; exit 2
  ;;
esac
