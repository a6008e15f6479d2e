#!/bin/bash
# Round-3 probe 2: k_reduce fast-path A/B (MOX_RED_KEYPROBE 0 / 1 / 2): parity
# of each variant on the reduce-heavy tests, then kernel averages in two
# interleaved rounds.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/p2; mkdir -p $O
step() { echo "== $1 rc=$2"; [ "$2" -eq 0 ] || exit "$2"; }
for v in kp1 kp2; do
  MOX_LIB=build/var_$v/libmox.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_exchange.py -x -q --timeout 200 \
    --timeout-method thread -k "kats or fuzz or corpora or split or high or exchange or dictionary" > $O/par_$v.log 2>&1
  step "parity $v $(tail -1 $O/par_$v.log)" $?
done
bash tools/ab_kernel.sh "base kp1 kp2" "0" "k_reduce k_map k_split_count" > $O/abk1.txt 2>&1; step "abk round 1" $?
cat $O/abk1.txt
bash tools/ab_kernel.sh "kp2 kp1 base" "0" "k_reduce k_map k_split_count" > $O/abk2.txt 2>&1; step "abk round 2" $?
cat $O/abk2.txt
