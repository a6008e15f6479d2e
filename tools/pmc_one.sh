#!/bin/bash
# One PMC pass (counters in $1) for kernel regex $2 over a bench run with args $3...
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
CTR=$1; K=$2; TAG=$3; shift 3
OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -s KILL 120 rocprofv3 --pmc $CTR --kernel-include-regex "$K" --output-format csv -d $OUT -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline "$@" > $OUT/log 2>&1
rc=$?; echo "$TAG rc=$rc"; [ $rc -eq 0 ] || { tail -5 $OUT/log; exit $rc; }
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
d = collections.defaultdict(list)
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        d[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in sorted(d.items()):
    print("%-32s %.4g (n=%d)" % (k, sorted(v)[len(v)//2], len(v)))
PY
