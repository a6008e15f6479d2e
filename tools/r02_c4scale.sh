#!/bin/bash
# k_reduce_small phase cycles (MOX_SR_STATS build) and kernel times at two C4 sizes.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/c4s; mkdir -p $O
for gb in 2 16; do
  MOX_VERBOSE=1 MOX_LIB=build/var_srstats/libmox.so timeout -k 10 300 python3 bench.py --workload C4 --bytes-per-gpu $((gb<<30)) \
    --steps 1 --warmup 1 --sync-passes --no-cpu-baseline > $O/st_$gb.json 2> $O/st_$gb.err
  rc=$?; echo "stats ${gb}G rc=$rc"; grep "dbg counters" $O/st_$gb.err | tail -1; [ $rc -eq 0 ] || exit $rc
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/p$gb -o run -- python3 bench.py --workload C4 \
    --bytes-per-gpu $((gb<<30)) --steps 2 --warmup 1 --no-cpu-baseline > $O/b_$gb.json 2> $O/b_$gb.err
  rc=$?; echo "trace ${gb}G rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
