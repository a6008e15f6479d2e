#!/bin/bash
# Interleaved A/B of libmox.so variants on the bench (build/var_NAME, see
# tools/build_variant.sh), after a quick parity check of every variant.
# Usage: bash tools/ab.sh "NAME1 NAME2 ..." ROUNDS [bench args...]
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
VARS=$1; ROUNDS=${2:-2}; shift 2
ARGS=${@:---steps 20 --warmup 5 --no-cpu-baseline}
O=gpurun_out/ab; mkdir -p $O
for v in $VARS; do
  MOX_LIB=build/var_$v/libmox.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 \
    --timeout-method thread -k "kats or fuzz or tile or corpora or huge or misaligned or split or async" > $O/par_$v.log 2>&1
  rc=$?; echo "parity $v rc=$rc $(tail -1 $O/par_$v.log)"; [ $rc -eq 0 ] || exit $rc
done
for r in $(seq $ROUNDS); do
  for v in $VARS; do
    MOX_LIB=build/var_$v/libmox.so timeout -k 10 200 python -u bench.py $ARGS > $O/b_${v}_$r.json 2> $O/b_${v}_$r.err
    rc=$?; [ $rc -eq 0 ] || { echo "bench $v rc=$rc"; tail -3 $O/b_${v}_$r.err; exit $rc; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], 'GB/s', d['value'], 'map_ms', d['roofline']['avg_launch_ms'], 'phases', d['phases_ms'])" $O/b_${v}_$r.json $v
  done
done
