#!/bin/bash
# Per-kernel A/B: rocprofv3 kernel-trace stats of the bench for each variant
# (build/var_NAME) and MOX_DBG value; prints the average duration of KERNELS.
# Usage: bash tools/ab_kernel.sh "NAME1 NAME2" "DBG1 DBG2" "k_reduce k_map" [bench args...]
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
VARS=$1; DBGS=$2; KS=$3; shift 3
ARGS=${@:---steps 10 --warmup 2 --no-cpu-baseline}
O=gpurun_out/abk; mkdir -p $O
for v in $VARS; do
  for d in $DBGS; do
    D=$O/${v}_$d
    MOX_LIB=build/var_$v/libmox.so MOX_DBG=$d timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $D -o run -- \
      python3 bench.py $ARGS > $D.log 2>&1
    rc=$?; [ $rc -eq 0 ] || { echo "$v dbg $d rc=$rc"; tail -3 $D.log; exit $rc; }
    python3 - "$D/run_kernel_stats.csv" "$v dbg=$d" "$D.log" $KS <<'PY'
import csv, json, sys
rows = {r["Name"].split("(")[0]: r for r in csv.DictReader(open(sys.argv[1]))}
gbs = ""
try:
    gbs = "%.1f GB/s " % json.loads(open(sys.argv[3]).read().strip().splitlines()[-1])["value"]
except Exception:
    pass
print(sys.argv[2], gbs + " ".join("%s %.1fus" % (k, float(rows[k]["AverageNs"]) / 1e3) for k in sys.argv[4:] if k in rows))
PY
  done
done
