#!/bin/bash
# k_map SQ instruction counts under the map ablations (build/abl = -DMOX_ABLATE):
# MOX_DBG 0 = full, 2 = byte phase + token list only (no token passes), 1 = no token list
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/pmcabl
for d in 0 2 1; do
  MOX_LIB=build/abl/libmox.so MOX_DBG=$d timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU,SQ_INSTS_SALU,SQ_INSTS_LDS,SQ_WAVE_CYCLES,SQ_WAIT_ANY,SQ_INSTS_BRANCH,SQ_ACTIVE_INST_VALU,SQ_WAIT_INST_ANY --kernel-include-regex "k_map" --output-format csv -d gpurun_out/pmcabl/d$d -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --sync-passes > gpurun_out/pmcabl/d$d.log 2>&1
  rc=$?; echo "dbg $d rc=$rc"; [ $rc -eq 0 ] || exit $rc
  python3 - gpurun_out/pmcabl/d$d <<'PY'
import csv, glob, sys, collections
d = collections.defaultdict(list)
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        d[r["Counter_Name"]].append(float(r["Counter_Value"]))
print("  " + "  ".join("%s=%.3g" % (k, sorted(v)[len(v)//2]) for k, v in sorted(d.items())))
PY
done
