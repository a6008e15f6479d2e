"""Per-phase averages of k_reduce's DBG_STAMP timestamps (gpurun_out/stamps.csv,
s_memrealtime at 100 MHz): streaming (wave 0), inserts drained, sort, write-out."""
import csv
import statistics
import sys

rows = [list(map(int, r)) for r in csv.reader(open(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/stamps.csv"))]
rows = [r for r in rows if r[1] and r[5]]
t0 = min(r[1] for r in rows)
ph = {"stream": [], "insert_tail": [], "sort": [], "write": [], "total": []}
for r in rows:
    _, a, b, c, d, e, hw, nu = r
    ph["stream"].append((b - a) / 100)
    ph["insert_tail"].append((c - b) / 100)
    ph["sort"].append((d - c) / 100)
    ph["write"].append((e - d) / 100)
    ph["total"].append((e - a) / 100)
print("%d partitions, span %.1f us" % (len(rows), (max(r[5] for r in rows) - t0) / 100))
for k, v in ph.items():
    print("%-12s mean %7.2f us  median %7.2f  max %7.2f" % (k, statistics.mean(v), statistics.median(v), max(v)))
print("uniques/partition mean %.0f" % statistics.mean(r[7] for r in rows))
