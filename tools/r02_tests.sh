#!/bin/bash
# Round-2 test evidence: the whole GPU suite including the slow full-size
# tests, then the exchange tests once more with a synchronisation after every
# launch (MOX_SYNC_EACH=1) under a rocprofv3 kernel trace.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r02t}; mkdir -p $O
timeout -k 10 420 python -u -m pytest tests -m "gpu and not slow" -v --timeout 300 --timeout-method thread > $O/gpu_fast.log 2>&1
rc=$?; echo "fast rc=$rc $(tail -1 $O/gpu_fast.log)"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests -m "gpu and slow" -v --timeout 580 --timeout-method thread > $O/gpu_slow.log 2>&1
rc=$?; echo "slow rc=$rc $(tail -1 $O/gpu_slow.log)"; [ $rc -eq 0 ] || exit $rc
MOX_SYNC_EACH=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/xsync -o run -- python3 -m pytest \
  tests/test_gpu_exchange.py -q --timeout 250 --timeout-method thread > $O/exchange_sync_each.log 2>&1
rc=$?; echo "exchange sync-each rc=$rc $(tail -1 $O/exchange_sync_each.log)"; exit $rc
