#!/bin/bash
# Round 4, GPU call B: C4 16 GiB kernel A/B of the round-3 kernels (var_base)
# against the QF-region layout (var_qf: k_map without a dictionary keeps 4
# regions per partition, k_split_scatter moves a partition slice by slice),
# then the k_map time ladder at C2 (tools/r04_ladder.sh).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-x2}; mkdir -p $O
step() { echo "== $1 rc=$2"; [ "$2" -eq 0 ] || exit "$2"; }
bash tools/ab_kernel.sh "base qfpair qf" "0" "k_map k_split_count k_split_scatter k_reduce_sort1 k_mat" --workload C4 --steps 3 --warmup 1 --no-cpu-baseline > $O/c4_ab.txt 2>&1; step "c4 ab" $?
cat $O/c4_ab.txt
for v in base qfpair qf; do grep -o '"value": [0-9.]*' gpurun_out/abk/${v}_0.log | head -1; done
bash tools/r04_ladder.sh > $O/ladder.txt 2>&1; step "ladder" $?
cat $O/ladder.txt
