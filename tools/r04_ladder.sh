#!/bin/bash
# Round 4: k_map time ladder at C2 (verdict r3 item 3).  An -DMOX_ABLATE build
# runs the bench under a rocprofv3 kernel trace with the MOX_DBG stages
#   4096 loader + ring only (consumers release rows untouched)
#      1 + byte phase (token-start masks, no list)
#      2 + token list (list + odd tokens, no token pass)
#     24 + token pass without dictionary adds and cold stores (probes only)
#      8 + dictionary adds (no cold stores)
#      0 full kernel
# and prints k_map's average launch time per stage (tools/ab_kernel.sh).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/ab_kernel.sh "abl" "4096 1 2 24 8 0" "k_map" --steps 10 --warmup 2 --no-cpu-baseline
