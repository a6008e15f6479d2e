#!/bin/bash
# Round-3 probe 7: k_map after the dictionary rework: SQ counters, per-row
# phase cycles (MOX_STAMP build).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/p7; mkdir -p $O/st
step() { echo "== $1 rc=$2"; [ "$2" -eq 0 ] || exit "$2"; }
MOX_LIB=build/var_stamp/libmox.so MOX_DBG=1024 MOX_DEBUG_DIR=$O/st timeout -k 10 200 python -u bench.py --steps 2 --warmup 1 \
  --no-cpu-baseline > $O/stamp.log 2>&1; step "stamp bench" $?
python3 tools/mapcyc.py $O/st/mapcyc.csv; step "mapcyc" $?
bash tools/pmc_sq.sh k_map p7/sqmap > $O/sqmap.txt 2>&1; step "sq k_map" $?
cat $O/sqmap.txt
