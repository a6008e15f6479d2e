#!/bin/bash
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
K=${1:-k_map}; OUT=gpurun_out/${2:-ic}; mkdir -p $OUT
timeout -s KILL 90 rocprofv3 --pmc SQC_ICACHE_MISSES,SQC_ICACHE_HITS,SQ_INSTS_VALU,SQ_INSTS_SALU,SQ_WAVE_CYCLES,SQ_WAIT_INST_ANY --kernel-include-regex "$K" --output-format csv -d $OUT/p1 -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > $OUT/p1.log 2>&1
rc=$?; echo "ic rc=$rc"; [ $rc -eq 0 ] || { tail -5 $OUT/p1.log; exit $rc; }
python3 - "$OUT/p1" <<'PY'
import csv, glob, sys, collections
d = collections.defaultdict(list)
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        d[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in d.items():
    print("%-24s %.4g (n=%d)" % (k, sorted(v)[len(v)//2], len(v)))
PY
