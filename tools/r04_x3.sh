#!/bin/bash
# Round 4, GPU call C: the engine-group / bytewise-sort GPU tests and the N = 2
# group bench on the bytewise sort v3, then call B's kernel A/Bs and the k_map
# ladder (tools/r04_x2.sh).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-x3}; mkdir -p $O
step() { echo "== $1 rc=$2"; [ "$2" -eq 0 ] || exit "$2"; }
timeout -k 10 400 python -u -m pytest tests/test_gpu_group.py tests/test_table_sort.py -x -v --timeout 200 --timeout-method thread -m "gpu and not slow" > $O/group_tests.log 2>&1; rc=$?; step "group tests $(tail -1 $O/group_tests.log)" $rc
timeout -k 10 400 python -u bench.py --gpus 2 --xport host --device 0 --steps 3 --warmup 1 > $O/n2.json 2> $O/n2.err; step "bench n2" $?
python3 -c "import json;d=json.load(open('$O/n2.json'));print(d['value'],d['phases_ms'])"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/n2t -o run -- python3 bench.py --gpus 2 --xport host --device 0 --steps 2 --warmup 1 > $O/n2t.json 2> $O/n2t.err; step "rocprof n2" $?
bash tools/r04_x2.sh ${1:-x3}
