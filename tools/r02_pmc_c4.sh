#!/bin/bash
# HBM traffic (FETCH_SIZE x2 / WRITE_SIZE, separate passes) of the C4 kernels.
set -o pipefail
for k in k_split_scatter k_reduce_sort1 k_map; do
  for c in FETCH_SIZE WRITE_SIZE; do
    bash tools/pmc_one.sh $c "^$k\$" pmc_c4_${k}_$c --workload C4 || exit $?
  done
done
