#!/bin/bash
# per-kernel time of the exchange benchmark (tools/xbench.py) under rocprofv3
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/xs; mkdir -p $OUT
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o run -- python3 tools/xbench.py > $OUT/log 2>&1
rc=$?; echo "rc=$rc"; grep "exchange" $OUT/log | tail -2
cut -d, -f1-4 $OUT/run_kernel_stats.csv
exit $rc
