#!/bin/bash
# SQ / traffic counters of several kernels (regex $1) over a bench run
# (BENCH_ARGS), one rocprofv3 pass per counter group, medians per kernel.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
K=$1; TAG=${2:-pmck}
OUT=gpurun_out/$TAG; mkdir -p $OUT
i=0
# PMC_GROUPS: space-separated counter groups instead of the four below
CGROUPS=${PMC_GROUPS:-"SQ_WAVES,SQ_INSTS_VALU,SQ_INSTS_SALU,SQ_INSTS_LDS,SQ_WAVE_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY \
SQ_INSTS_VMEM_RD,SQ_INSTS_VMEM_WR,SQ_LDS_BANK_CONFLICT,SQ_ACTIVE_INST_VALU,SQ_ACTIVE_INST_LDS,SQ_BUSY_CYCLES,SQ_WAIT_INST_LDS,SQ_INST_CYCLES_VMEM \
FETCH_SIZE WRITE_SIZE,GRBM_GUI_ACTIVE"}
for grp in $CGROUPS; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $grp --kernel-include-regex "$K" --output-format csv -d $OUT/p$i -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline ${BENCH_ARGS} > $OUT/p$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"; [ $rc -eq 0 ] || { tail -5 $OUT/p$i.log; exit $rc; }
done
python3 - "$OUT" <<'PY' | tee $OUT/summary.txt
import csv, glob, sys, collections
d = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(sys.argv[1] + "/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        d[r["Kernel_Name"].split("(")[0]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k in sorted(d):
    print("==", k)
    for c, v in sorted(d[k].items()):
        v = sorted(v)
        print("  %-28s %.5g (n=%d, max %.5g)" % (c, v[len(v)//2], len(v), v[-1]))
PY
