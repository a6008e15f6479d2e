"""Mean per-wave cycles of k_reduce's streaming loop by segment (MOX_RED_STATS
build, MOX_DBG=1024): gpurun_out/redcyc.csv rows = wave, [0] between chunks
(loop, load issue), [1] data wait + hash, [2] fast path, [3] slow path."""
import csv
import sys

rows = [list(map(int, r)) for r in csv.reader(open(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/redcyc.csv"))]
rows = [r for r in rows if sum(r[1:])]
n = len(rows)
names = ["between", "wait+hash", "fast", "slow"]
tot = [sum(r[k + 1] for r in rows) / n for k in range(4)]
print("%d waves; mean cycles per wave: " % n + ", ".join("%s %.0f" % (a, b) for a, b in zip(names, tot)) + ", sum %.0f" % sum(tot))
