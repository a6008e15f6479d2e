#!/bin/bash
# End-to-end bench A/B of build variants (build/var_NAME), interleaved: value, ms/step, k_map ms per line.
set -o pipefail
mkdir -p gpurun_out/${AB_TAG:-bab}
for v in ${AB_VARS:-sd0 sd1 sd0 sd1}; do
  MOX_LIB=build/var_$v/libmox.so timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 20 --warmup 20 > gpurun_out/${AB_TAG:-bab}/$v.json 2> gpurun_out/${AB_TAG:-bab}/$v.err || { echo "$v failed"; exit 1; }
  python3 -c "import json,sys;d=json.loads(open('gpurun_out/${AB_TAG:-bab}/$v.json').read().strip().splitlines()[-1]);print('$v', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'])" | tee -a gpurun_out/${AB_TAG:-bab}/ab.txt
done
