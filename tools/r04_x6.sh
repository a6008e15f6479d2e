#!/bin/bash
# Round 4, GPU call F: k_map loader row-group batch A/B at C2 (var_ldr: row by row,
# var_ldb: one poll, write and publish per row group), interleaved
# twice; the k_map time ladder with the fenced loader; the C2 bench line.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-x5}; mkdir -p $O
step() { echo "== $1 rc=$2"; [ "$2" -eq 0 ] || exit "$2"; }
bash tools/ab_kernel.sh "ldr ldb ldr ldb" "0" "k_map k_reduce" > $O/ldb_ab.txt 2>&1; rc=$?; cat $O/ldb_ab.txt; step "ldb ab" $rc
for v in ldr ldb; do echo "$v $(grep -o '"value": [0-9.]*' gpurun_out/abk/${v}_0.log | head -1)"; done
bash tools/r04_ladder.sh > $O/ladder.txt 2>&1; rc=$?; cat $O/ladder.txt; step "ladder" $rc
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/bench_c2.json 2> $O/bench_c2.err; step "bench C2" $?
python3 -c "import json;d=json.loads(open('$O/bench_c2.json').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'],d['roofline']['avg_launch_ms'],d['phases_ms'])"
