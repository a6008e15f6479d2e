#!/bin/bash
# k_map SQ instruction counts per MOX_DBG ablation stage of a -DMOX_ABLATE build
# (build/var_$VAR, default abl): VALU / SALU / LDS / branch instructions and
# VALU-active quad-cycles per launch, and per 992-byte row.
# Usage: bash tools/pmc_map_stages.sh TAG "STAGES"   (e.g. "4096 1 2 8 0")
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${1:-stages}; STAGES=${2:-4096 1 2 0}; VAR=${VAR:-abl}; KRE=${KRE:-k_map}; UNITS=${UNITS:-1082402}
O=gpurun_out/$TAG; mkdir -p $O
for d in $STAGES; do
  MOX_LIB=build/var_$VAR/libmox.so MOX_DBG=$d timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU,SQ_INSTS_SALU,SQ_INSTS_LDS,SQ_INSTS_BRANCH,SQ_ACTIVE_INST_VALU,SQ_WAVE_CYCLES,SQ_WAIT_ANY,SQ_INSTS_SMEM \
    --kernel-include-regex "$KRE" --output-format csv -d $O/d$d -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --sync-passes > $O/d$d.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "dbg $d rc=$rc"; tail -3 $O/d$d.log; exit $rc; }
  python3 - $O/d$d $d $UNITS <<'PY'
import csv, glob, sys, collections
d = collections.defaultdict(list)
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        d[r["Counter_Name"]].append(float(r["Counter_Value"]))
m = {k: sorted(v)[len(v) // 2] for k, v in d.items()}
rows = float(sys.argv[3])  # per-unit divisor: C2 rows per launch (1 GiB / 992 B) by default; KRE/UNITS for other kernels
print("dbg %-5s " % sys.argv[2] + "  ".join("%s %.1f/row" % (k.replace("SQ_", ""), v / rows) for k, v in sorted(m.items())))
PY
done
