#!/bin/bash
# Address-translation and read-latency counters of one kernel per build
# variant and MOX_DBG stage: UTCL1 hits / misses and the TCP->TCC read
# latency per request (one --pmc pass each, 4 TCP counters).
# Usage: bash tools/pmc_tlb.sh TAG "VAR:DBG ..." KERNEL_REGEX
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=$1; RUNS=$2; KRE=$3
O=gpurun_out/$TAG; mkdir -p $O
for vd in $RUNS; do
  v=${vd%%:*}; d=${vd##*:}
  MOX_LIB=build/var_$v/libmox.so MOX_DBG=$d timeout -s KILL 90 rocprofv3 --pmc TCP_UTCL1_TRANSLATION_MISS_sum,TCP_UTCL1_TRANSLATION_HIT_sum,TCP_TCC_READ_REQ_LATENCY_sum,TCP_TCC_READ_REQ_sum \
    --kernel-include-regex "$KRE" --output-format csv -d $O/${v}_$d -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --sync-passes > $O/${v}_$d.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "$vd rc=$rc"; tail -n 3 $O/${v}_$d.log; exit $rc; }
  python3 - $O/${v}_$d $vd <<'PY'
import csv, glob, sys, collections
d = collections.defaultdict(list)
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        d[r["Counter_Name"]].append(float(r["Counter_Value"]))
m = {k: sorted(v)[len(v) // 2] for k, v in d.items()}
g = lambda k: m.get(k, float("nan"))
print("%-12s" % sys.argv[2], "  ".join("%s %.4g" % (k, v) for k, v in sorted(m.items())),
      " miss/(hit+miss) %.3f  read latency %.0f cyc/req" % (g("TCP_UTCL1_TRANSLATION_MISS_sum") / max(1, g("TCP_UTCL1_TRANSLATION_MISS_sum") + g("TCP_UTCL1_TRANSLATION_HIT_sum")),
                                                          g("TCP_TCC_READ_REQ_LATENCY_sum") / max(1, g("TCP_TCC_READ_REQ_sum"))))
PY
done
