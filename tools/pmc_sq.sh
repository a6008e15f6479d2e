#!/bin/bash
# SQ instruction-mix / stall / LDS counters for one kernel (one pass per counter group)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
K=${1:-k_map}; TAG=${2:-sq}
OUT=gpurun_out/$TAG; mkdir -p $OUT
i=0
for grp in "SQ_WAVES,SQ_INSTS_VALU,SQ_INSTS_SALU,SQ_INSTS_LDS,SQ_WAVE_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY" \
           "SQ_INSTS_VMEM_RD,SQ_INSTS_VMEM_WR,SQ_LDS_BANK_CONFLICT,SQ_ACTIVE_INST_VALU,SQ_ACTIVE_INST_LDS,SQ_INST_CYCLES_VMEM,SQ_WAIT_INST_LDS,SQ_BUSY_CYCLES" \
           "SQ_LDS_IDX_ACTIVE,SQ_LDS_ADDR_CONFLICT,SQ_LDS_UNALIGNED_STALL,SQ_INSTS_BRANCH,SQ_ACTIVE_INST_SCA,SQ_INSTS_SMEM,SQ_IFETCH,SQ_ACTIVE_INST_MISC" \
           "GRBM_GUI_ACTIVE,GRBM_COUNT"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp --kernel-include-regex "$K" --output-format csv -d $OUT/p$i -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline ${BENCH_ARGS} > $OUT/p$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"; [ $rc -eq 0 ] || { tail -5 $OUT/p$i.log; exit $rc; }
  python3 - "$OUT/p$i" <<'PY'
import csv, glob, sys, collections
d = collections.defaultdict(list)
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        d[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in d.items():
    print("%-24s %.4g (n=%d)" % (k, sorted(v)[len(v)//2], len(v)))
PY
done
