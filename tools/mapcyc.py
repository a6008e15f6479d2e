"""Per-row phase cycles of k_map's consumer waves from a -DMOX_STAMP build
(mapcyc.csv under $MOX_DEBUG_DIR: wave, wait, byte+list, token pass, the
counted row-DMA wait inside "wait" (MOX_MAP_SELF builds), -, rows, finish): cycles per row per phase, averaged over the consumer waves."""
import csv
import sys

rows = [list(map(int, r)) for r in csv.reader(open(sys.argv[1] if len(sys.argv) > 1 else "mapcyc.csv"))]
rows = [r for r in rows if r[6] > 0]
n = sum(r[6] for r in rows)
for name, k in (("wait", 1), ("byte+list", 2), ("token pass", 3), ("(vm wait)", 4)):
    print("%-11s %7.0f cycles/row" % (name, sum(r[k] for r in rows) / n))
print("rows %d over %d consumer waves; total %.0f cycles/row" % (n, len(rows), sum(r[1] + r[2] + r[3] for r in rows) / n))
