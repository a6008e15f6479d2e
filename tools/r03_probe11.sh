#!/bin/bash
# Round-3 probe 11: fixed-capacity split scatter (no k_split_count histogram
# pass): split / collision tests on the current build, C4 16 GiB kernel
# averages and bench lines head vs fixcap.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/p11; mkdir -p $O
step() { echo "== $1 rc=$2"; [ "$2" -eq 0 ] || exit "$2"; }
timeout -k 10 500 python -u -m pytest tests/test_gpu_collide.py tests/test_gpu_parity.py tests/test_gpu_exchange.py tests/test_gpu_group.py -x -q \
  --timeout 300 --timeout-method thread -k "collide or split or high or hc or mixed or exchange or group or kats" > $O/par.log 2>&1; rc=$?; step "parity $(tail -1 $O/par.log)" $rc
timeout -k 10 400 python -u -m pytest tests/test_gpu_scale.py -x -q --timeout 380 --timeout-method thread -k "4gib" > $O/c4_4gib.log 2>&1; rc=$?; step "C4 4 GiB digest $(tail -1 $O/c4_4gib.log)" $rc
bash tools/ab_kernel.sh "head fixcap" "0" "k_split_count k_split_scatter k_reduce_sort1 k_map k_mat" --workload C4 --steps 2 --warmup 1 --no-cpu-baseline > $O/abk.txt 2>&1; step "abk C4" $?
cat $O/abk.txt
for v in head fixcap; do
  MOX_LIB=build/var_$v/libmox.so timeout -k 10 300 python -u bench.py --workload C4 --steps 5 --warmup 2 --no-cpu-baseline > $O/b_$v.json 2> $O/b_$v.err; step "bench C4 $v" $?
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], d['phases_ms'])" $O/b_$v.json $v
done
