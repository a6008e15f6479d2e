#!/bin/bash
# Round 4: (1) C4 k_map pair stores at consecutive addresses vs the regions
# (-DMOX_ABLATE 32768 / 0); (2) k_reduce ticket table + early ticket
# (build/var_cur) against the committed kernels (build/var_head), interleaved;
# (3) C4 batched pair protocol (build/var_pb0: -DMOX_PAIR_BATCH=0) against cur;
# (4) k_reduce stream-only time with the table (abl 64).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-x9}; mkdir -p $O
bash tools/ab_kernel.sh "abl" "32768 0" "k_map" --workload C4 --steps 3 --warmup 1 --no-cpu-baseline > $O/c4_seq.txt 2>&1; rc=$?
cat $O/c4_seq.txt; [ $rc -eq 0 ] || exit $rc
bash tools/ab_kernel.sh "pb0 cur pb0 cur" "0" "k_map" --workload C4 --steps 3 --warmup 1 --no-cpu-baseline > $O/c4_pb.txt 2>&1; rc=$?
cat $O/c4_pb.txt; [ $rc -eq 0 ] || exit $rc
bash tools/ab_kernel.sh "head cur head cur" "0" "k_reduce k_map" > $O/red_ab.txt 2>&1; rc=$?
cat $O/red_ab.txt; [ $rc -eq 0 ] || exit $rc
bash tools/ab_kernel.sh "abl" "64 0" "k_reduce" > $O/red_abl.txt 2>&1; rc=$?
cat $O/red_abl.txt; exit $rc
