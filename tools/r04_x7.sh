#!/bin/bash
# Round 4: where C4's k_map and C2's k_reduce spend their time (-DMOX_ABLATE
# build, tools/ab_kernel.sh), then a production C4 bench line.
#   C4 k_map stages: 4096 loader + ring only, 2 + token list, 8 + token pass
#   without cold stores (no pair protocol, no stores), 0 full
#   C2 k_reduce: 0 full, 64 no inserts (stream + hash), 128 no slow path,
#   512 plain (non-atomic) count add, 32 no sort
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-x7}; mkdir -p $O
bash tools/ab_kernel.sh "abl" "4096 2 8 0" "k_map k_split_count k_split_scatter k_reduce_sort1 k_mat" --workload C4 --steps 3 --warmup 1 --no-cpu-baseline > $O/c4_ladder.txt 2>&1; rc=$?
cat $O/c4_ladder.txt; [ $rc -eq 0 ] || exit $rc
bash tools/ab_kernel.sh "abl" "0 64 128 512 32" "k_reduce k_map" > $O/c2_red_abl.txt 2>&1; rc=$?
cat $O/c2_red_abl.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --workload C4 --steps 5 --warmup 2 --no-cpu-baseline > $O/bench_c4.json 2> $O/bench_c4.err; rc=$?
echo "== bench C4 rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 -c "
import json; l=json.load(open('$O/bench_c4.json')); print(l['value'], l['ms_per_step'], l['phases_ms'])"
