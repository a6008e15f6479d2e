#!/bin/bash
# Round 4, GPU call B (kernel A/Bs from rocprofv3 kernel traces, tools/ab_kernel.sh):
#  1. C4 16 GiB: round-3 kernels (var_base) vs the QF-region layout with paired
#     split writes (var_qfpair) vs LDS-staged slices (var_qf) vs var_qf with
#     k_reduce_sort1 at 3 workgroups per CU (var_s1w3: no VGPR spills);
#  2. C2: k_reduce with static wave shares (var_rstat) vs chunk tickets (var_qf);
#  3. the k_map time ladder at C2 (tools/r04_ladder.sh).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-x2}; mkdir -p $O
step() { echo "== $1 rc=$2"; [ "$2" -eq 0 ] || exit "$2"; }
bash tools/ab_kernel.sh "base qfpair qf s1w3" "0" "k_map k_split_count k_split_scatter k_reduce_sort1 k_reduce k_mat" --workload C4 --steps 3 --warmup 1 --no-cpu-baseline > $O/c4_ab.txt 2>&1; rc=$?; cat $O/c4_ab.txt; step "c4 ab" $rc
for v in base qfpair qf s1w3; do echo "$v $(grep -o '"value": [0-9.]*' gpurun_out/abk/${v}_0.log | head -1)"; done
bash tools/ab_kernel.sh "rstat qf rhome rstat qf rhome" "0" "k_map k_reduce" > $O/c2_red_ab.txt 2>&1; rc=$?; cat $O/c2_red_ab.txt; step "c2 reduce ab" $rc
bash tools/r04_ladder.sh > $O/ladder.txt 2>&1; rc=$?; cat $O/ladder.txt; step "ladder" $rc
