#!/bin/bash
# Round 4, GPU call A: the fast GPU suite on this tree, the C2 bench line, and
# a kernel + copy + HIP API trace of the N = 2 engine group (2 x 8 GiB C3
# shards, device-copy transport, both members on GPU 0) to account for the
# exchange phase (tools/step_timeline.py).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-x1}; mkdir -p $O
step() { echo "== $1 rc=$2"; [ "$2" -eq 0 ] || exit "$2"; }
timeout -k 10 700 python -u -m pytest tests -x -v --timeout 200 --timeout-method thread -m "gpu and not slow" > $O/gpu_fast.log 2>&1; rc=$?; step "gpu fast $(tail -1 $O/gpu_fast.log)" $rc
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/bench_c2.json 2> $O/bench_c2.err; step "bench C2" $?
cut -c1-160 $O/bench_c2.json
timeout -k 10 400 python -u bench.py --gpus 2 --xport host --device 0 --steps 3 --warmup 1 > $O/n2.json 2> $O/n2.err; step "bench n2" $?
python3 -c "import json;d=json.load(open('$O/n2.json'));print(d['value'],d['phases_ms'],d['hash_order'])"
timeout -k 10 500 rocprofv3 --kernel-trace --memory-copy-trace --hip-runtime-trace --output-format csv -d $O/n2t -o run -- \
  python3 bench.py --gpus 2 --xport host --device 0 --steps 2 --warmup 1 > $O/n2t.json 2> $O/n2t.err; step "rocprof n2" $?
python3 tools/step_timeline.py $O/n2t 30 > $O/n2_timeline.txt; step "timeline" $?
tail -3 $O/n2_timeline.txt
MOX_LIB=build/var_os8/libmox.so timeout -k 10 400 python -u bench.py --gpus 2 --xport host --device 0 --steps 3 --warmup 1 > $O/n2_os8.json 2> $O/n2_os8.err; step "bench n2 os8" $?
python3 -c "import json;d=json.load(open('$O/n2_os8.json'));print('os8',d['value'],d['phases_ms'])"
