#!/bin/bash
# Round 4, GPU call D: engine-group / sort GPU tests and the N = 2 bench on the
# bytewise sort v4 (packed run flags, LDS segmented run sort), a rocprofv3
# kernel trace of it; C4 16 GiB kernel A/B paired-split (var_qfpair) vs
# LDS-staged slices (var_qf), interleaved twice; the k_map time ladder.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-x4}; mkdir -p $O
step() { echo "== $1 rc=$2"; [ "$2" -eq 0 ] || exit "$2"; }
timeout -k 10 400 python -u -m pytest tests/test_gpu_group.py tests/test_table_sort.py -x -v --timeout 200 --timeout-method thread -m "gpu and not slow" > $O/group_tests.log 2>&1; rc=$?; step "group tests $(tail -1 $O/group_tests.log)" $rc
timeout -k 10 400 python -u bench.py --gpus 2 --xport host --device 0 --steps 3 --warmup 1 > $O/n2.json 2> $O/n2.err; step "bench n2" $?
python3 -c "import json;d=json.load(open('$O/n2.json'));print(d['value'],d['phases_ms'])"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/n2t -o run -- python3 bench.py --gpus 2 --xport host --device 0 --steps 2 --warmup 1 > $O/n2t.json 2> $O/n2t.err; step "rocprof n2" $?
bash tools/r04_ladder.sh > $O/ladder.txt 2>&1; rc=$?; cat $O/ladder.txt; step "ladder" $rc
bash tools/ab_kernel.sh "qfpair qf qfpair qf" "0" "k_map k_split_count k_split_scatter k_reduce_sort1 k_mat" --workload C4 --steps 3 --warmup 1 --no-cpu-baseline > $O/c4_ab.txt 2>&1; rc=$?; cat $O/c4_ab.txt; step "c4 ab" $rc
