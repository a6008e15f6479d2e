#!/bin/bash
# Round-6 GPU runs, one or more sections per call; every file under profiles/r06/
# names the section that produced it.  Usage on a GPU box (through gpurun):
#   bash tools/r06_runs.sh TAG SECTION [SECTION ...]     (outputs under gpurun_out/TAG)
#
# Sections:
#   fast     the fast GPU suite (gpu and not slow)
#   parity   the parity subset (test_gpu_parity, test_gpu_collide, test_gpu_exchange; not slow)
#   slow     the slow GPU tests
#   evid     default C2 bench line (with the CPU baseline), then a rocprofv3 kernel
#            trace + stats of the C2 bench and one pass's timeline
#   n2       N = 2 engine-group bench line (2 x 8 GiB C3 shards on GPU 0, sorted result,
#            same-work N = 1 figure), then a kernel + HIP API trace of the same command's
#            steps and the last step's timeline
#   lines    bench lines of C5 and C4 (16 GiB each)
#   ab       interleaved per-kernel A/B of build variants: AB_VARS="v1 v2 v1 v2"
#            AB_KERNELS="k_map" [AB_DBG="0"] [AB_ARGS="--workload C4 ..."]
#   abe      interleaved end-to-end bench A/B of variants: AB_VARS, AB_ARGS
#   sort     the device bytewise sort's GPU tests (group, exchange)
#   xsort    the exchange and engine-group GPU tests (not slow)
#   evab     bench line with / without the k_map timing events (interleaved)
#   overlap  tools/overlap_probe.py: one engine's async C2 passes vs two engines' at once
#   c2       the C2 bench line without the CPU baseline (value, k_map, sorted-result line)
#   c2prof   rocprofv3 kernel stats of that bench line (sort kernels)
#   varpar   a build variant (VAR=name: build/var_name) through the parity subset and the
#            full-size C2 async parity test
#   pmc      k_map FETCH/WRITE traffic at C2 and SQ counters of k_map
#   smoke    __graft_entry__.smoke()
#   abn2     interleaved N = 2 engine-group bench lines of build variants (AB_VARS)
#   n2prof   kernel trace of an N = 2 group bench (VAR=name) and the exchange reduce passes' kernels
#   abs      interleaved C2 bench lines of build variants (AB_VARS): value and the sorted-result line
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=$1; shift
O=gpurun_out/$TAG; mkdir -p $O
step() { echo "== $1 rc=$2"; [ "$2" -eq 0 ] || exit "$2"; }
pyt() {  # pyt LOG TIMEOUT pytest-args...
  local log=$1 to=$2; shift 2
  timeout -k 10 $to python -u -m pytest -x -v --timeout 300 --timeout-method thread "$@" > $O/$log 2>&1
  local rc=$?; step "$log $(tail -1 $O/$log)" $rc
}
for SEC in "$@"; do
case $SEC in
fast)
  pyt gpu_fast.log 900 tests -m "gpu and not slow"
  ;;
parity)
  pyt parity.log 700 tests/test_gpu_parity.py tests/test_gpu_collide.py tests/test_gpu_exchange.py -m "gpu and not slow"
  ;;
slow)
  pyt gpu_slow.log 1100 tests -m "gpu and slow"
  ;;
smoke)
  timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1
  step "smoke $(tail -1 $O/smoke.log)" $?
  ;;
evid)
  timeout -k 10 400 python -u bench.py > $O/bench_c2.json 2> $O/bench_c2.err; step "bench C2" $?
  cut -c1-300 $O/bench_c2.json
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c2 -o run -- \
    python3 bench.py --no-cpu-baseline > $O/c2_under_rocprof.log 2>&1; step "rocprof C2" $?
  python3 tools/trace_timeline.py $O/c2 > $O/c2_timeline.txt; step "timeline C2" $?
  tail -1 $O/c2_timeline.txt
  ;;
n2)
  timeout -k 10 500 python -u bench.py --gpus 2 --xport host --device 0 --steps 5 --warmup 2 > $O/bench_n2.json 2> $O/bench_n2.err
  step "bench N2 group" $?
  cut -c1-300 $O/bench_n2.json
  timeout -k 10 500 rocprofv3 --kernel-trace --hip-trace --memory-copy-trace --output-format csv -d $O/n2tr -o run -- \
    python3 bench.py --gpus 2 --xport host --device 0 --steps 3 --warmup 1 > $O/n2_under_rocprof.log 2>&1; step "rocprof N2" $?
  python3 tools/step_timeline.py $O/n2tr 30 > $O/n2_step_timeline.txt; step "step timeline N2" $?
  tail -3 $O/n2_step_timeline.txt
  ;;
abn2)
  # interleaved N = 2 engine-group bench lines of build variants: AB_VARS="v1 v2 v1 v2"
  k=0
  for v in $AB_VARS; do
    k=$((k+1)); f=$O/abn2_${k}_${v}
    MOX_LIB=build/var_$v/libmox.so timeout -k 10 400 python -u bench.py --gpus 2 --xport host --device 0 --steps 5 --warmup 2 > $f.json 2> $f.err
    rc=$?; [ $rc -eq 0 ] || { tail -3 $f.err; step "abn2 $v" $rc; }
    python3 -c "import json;d=json.loads(open('$f.json').read().strip().splitlines()[-1]);m=d['multi_gpu'];h=d['hash_order'];print('$v', d['value'], 'exchange', m['exchange_ms'], 'sort', d['phases_ms']['sort_bytes'], 'hash', h['value'], h['phases_ms']['exchange'])"
  done
  ;;
n2prof)
  # kernel trace of an N = 2 group bench (VAR=name: build/var_name), the exchange reduce passes' kernels
  L=${VAR:+build/var_$VAR/libmox.so}; L=${L:-map-oxidize_amd/mox/libmox.so}
  MOX_LIB=$L timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/n2k_${VAR:-tree} -o run -- \
    python3 bench.py --gpus 2 --xport host --device 0 --steps 3 --warmup 1 > $O/n2k_${VAR:-tree}.log 2>&1; step "rocprof N2 ${VAR:-tree}" $?
  python3 tools/xpass_kernels.py $O/n2k_${VAR:-tree} > $O/xpass_${VAR:-tree}.txt; step "xpass ${VAR:-tree}" $?
  cat $O/xpass_${VAR:-tree}.txt
  ;;
abs)
  # interleaved C2 bench lines of build variants (AB_VARS): value and the sorted-result line
  k=0
  for v in $AB_VARS; do
    k=$((k+1)); f=$O/abs_${k}_${v}
    MOX_LIB=build/var_$v/libmox.so timeout -k 10 300 python -u bench.py --no-cpu-baseline ${AB_ARGS:-} > $f.json 2> $f.err
    rc=$?; [ $rc -eq 0 ] || { tail -3 $f.err; step "abs $v" $rc; }
    python3 -c "import json;d=json.loads(open('$f.json').read().strip().splitlines()[-1]);s=d['sorted_result'];print('$v', d['value'], 'sorted', s['value'], 'sort_ms', s.get('sort_bytes_ms'))"
  done
  ;;
lines)
  timeout -k 10 420 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --workload C5 > $O/bench_c5.json 2> $O/bench_c5.err; step "bench C5" $?
  cut -c1-200 $O/bench_c5.json
  timeout -k 10 600 python -u bench.py --steps 3 --warmup 2 --no-cpu-baseline --workload C4 > $O/bench_c4.json 2> $O/bench_c4.err; step "bench C4" $?
  cut -c1-200 $O/bench_c4.json
  ;;
ab)
  bash tools/ab_kernel.sh "$AB_VARS" "${AB_DBG:-0}" "$AB_KERNELS" ${AB_ARGS:-} > $O/ab.txt 2>&1; rc=$?; cat $O/ab.txt; step ab $rc
  ;;
abe)
  # a spec is NAME or NAME@PIECES (--sample-pieces PIECES); every run of a spec is kept (suffix _k)
  k=0
  for spec in $AB_VARS; do
    k=$((k+1)); v=${spec%@*}; sp=""; [ "$spec" != "$v" ] && sp="--sample-pieces ${spec#*@}"
    f=$O/abe_${k}_${v}
    MOX_LIB=build/var_$v/libmox.so timeout -k 10 300 python -u bench.py --no-cpu-baseline $sp ${AB_ARGS:-} > $f.json 2> $f.err
    rc=$?; [ $rc -eq 0 ] || { tail -3 $f.err; step "abe $spec" $rc; }
    python3 -c "import json,sys;d=json.loads(open('$f.json').read().strip().splitlines()[-1]);print('$spec', d['value'], d['roofline']['avg_launch_ms'], d['stats']['cold_records'], d['stats']['dict_words'])"
  done
  ;;
sort)
  # the device bytewise sort: its own tests, the sorted exchange, the group's sorted table
  pyt sort.log 600 tests/test_gpu_group.py tests/test_gpu_exchange.py -m "gpu and not slow" -k "sort"
  ;;
xsort)
  # the exchange and engine-group tests (sorted exchange, device splitters, device sort)
  pyt xsort.log 900 tests/test_gpu_exchange.py tests/test_gpu_group.py -m "gpu and not slow"
  ;;
evab)
  # the k_map timing events' cost: the default bench line against the same
  # steps without events around k_map, interleaved
  for k in 1 2; do
    for v in ev noev; do
      f=$O/evab_${k}_$v.json; x=""; [ $v = noev ] && x="--no-map-events"
      timeout -k 10 300 python -u bench.py --no-cpu-baseline $x > $f 2> $O/evab_${k}_$v.err; step "evab $k $v" $?
      python3 -c "import json;d=json.loads(open('$f').read().strip().splitlines()[-1]);print('$v', d['value'], d['ms_per_step'])"
    done
  done
  ;;
overlap)
  timeout -k 10 400 python -u tools/overlap_probe.py 30 20 > $O/overlap.txt 2>&1; step "overlap probe" $?
  cat $O/overlap.txt
  ;;
c2)
  timeout -k 10 400 python -u bench.py --no-cpu-baseline > $O/bench_c2.json 2> $O/bench_c2.err; step "bench C2" $?
  python3 -c "import json;d=json.loads(open('$O/bench_c2.json').read().strip().splitlines()[-1]);print(d['value'], d['roofline']['avg_launch_ms'], d['sorted_result'])"
  ;;
c2prof)
  # rocprofv3 kernel stats of the C2 bench (no CPU baseline): the sort kernels' averages
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c2p -o run -- \
    python3 bench.py --no-cpu-baseline > $O/c2p_under_rocprof.log 2>&1; step "rocprof C2" $?
  f=$(ls $O/c2p/*/run_kernel_stats.csv 2>/dev/null | head -1); [ -n "$f" ] || f=$(ls $O/c2p/run_kernel_stats.csv)
  cut -d, -f1-4 "$f" | grep -E "k_ss_|k_os_pass|k_bs_|k_scan|k_map|k_reduce\"" ; true
  python3 tools/sort_timeline.py $O/c2p > $O/sort_timeline.txt; step "sort timeline" $?
  tail -1 $O/sort_timeline.txt
  ;;
varpar)
  # a build variant (build/var_$VAR) through the parity subset and the full-size
  # C2 async bench-mode parity test
  MOX_LIB=build/var_${VAR}/libmox.so pyt varpar_$VAR.log 700 tests/test_gpu_parity.py tests/test_gpu_exchange.py -m "gpu and not slow"
  MOX_LIB=build/var_${VAR}/libmox.so pyt varc2_$VAR.log 400 tests/test_gpu_scale.py -m gpu -k "async_bench_mode"
  ;;
pmc)
  bash tools/pmc_traffic_wl.sh C2 1073741824 ${TAG}_traffic > $O/traffic.txt 2>&1; rc=$?; tail -5 $O/traffic.txt; step traffic $rc
  bash tools/pmc_sq.sh k_map ${TAG}_sqmap > $O/sq_k_map.txt 2>&1; rc=$?; cat $O/sq_k_map.txt; step "sq k_map" $rc
  ;;
*)
  echo "unknown section $SEC"; exit 2
  ;;
esac
done
