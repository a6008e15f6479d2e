#!/bin/bash
# k_reduce cycle accounting (MOX_RED_STATS build) + phase stamps + slow-path
# counters, and the ingest probe (tools/ingest_probe.cpp).
set -e
mkdir -p gpurun_out/rst
MOX_LIB=build/var_rst/libmox.so MOX_DBG=$((1024+256)) MOX_DEBUG_DIR=gpurun_out/rst timeout -k 10 120 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --sync-passes > gpurun_out/rst/b.log 2> gpurun_out/rst/b.err
grep "dbg_cnt" gpurun_out/rst/b.err | tail -2
python tools/redcyc.py gpurun_out/rst/redcyc.csv
python tools/stamps.py gpurun_out/rst/stamps.csv
if [ -n "$INGEST" ]; then timeout -k 10 200 build/ingest_probe /tmp/ingest_probe.bin 1024; fi
