#!/bin/bash
# Round-2 GPU evidence run: slow full-size tests, bench lines for C2 / C4 / C5
# (CPU baseline median of 3), the N = 2 bench path (two ranks sharing GPU 0
# over the host transport), and the C4 kernel-stats profile.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r02a
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_scale.py tests/test_gpu_parity.py::test_full_size_c2 -x -v \
  --timeout 600 --timeout-method thread > $O/slow.log 2>&1
rc=$?; echo "slow tests rc=$rc"; tail -6 $O/slow.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py > $O/bench_c2.json 2> $O/bench_c2.err
rc=$?; echo "bench C2 rc=$rc"; cut -c1-400 $O/bench_c2.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 420 python -u bench.py --workload C4 --steps 5 --warmup 2 --cpu-sample-mib 256 > $O/bench_c4.json 2> $O/bench_c4.err
rc=$?; echo "bench C4 rc=$rc"; cut -c1-400 $O/bench_c4.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 420 python -u bench.py --workload C5 --steps 5 --warmup 2 --cpu-sample-mib 1024 > $O/bench_c5.json 2> $O/bench_c5.err
rc=$?; echo "bench C5 rc=$rc"; cut -c1-400 $O/bench_c5.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29571 \
  bench.py --gpus 2 --steps 5 --warmup 2 --xport host --device 0 --bytes-per-gpu 1073741824 > $O/bench_n2host.json 2> $O/bench_n2host.err
rc=$?; echo "bench N2 host rc=$rc"; cut -c1-600 $O/bench_n2host.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c4 -o run -- python3 bench.py --workload C4 \
  --steps 3 --warmup 1 --no-cpu-baseline > $O/prof_c4.log 2>&1
rc=$?; echo "rocprof C4 rc=$rc"; cut -d, -f1-4 $O/prof_c4/run_kernel_stats.csv | head -30
exit $rc
