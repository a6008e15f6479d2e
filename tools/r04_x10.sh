#!/bin/bash
# Round 4: k_reduce per-partition phase stamps at C2 (-DMOX_ABLATE, DBG_STAMP
# = 1024; tools/stamps.py): full inserts, and streaming without inserts (1088).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-x10}; mkdir -p $O
for d in 1024 1088; do
  mkdir -p $O/s$d
  MOX_LIB=build/var_abl/libmox.so MOX_DBG=$d MOX_DEBUG_DIR=$O/s$d timeout -k 10 200 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/s$d.log 2>&1; rc=$?
  [ $rc -eq 0 ] || { tail -5 $O/s$d.log; exit $rc; }
  echo "== dbg $d"; python3 tools/stamps.py $O/s$d/stamps.csv
done
