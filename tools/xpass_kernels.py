"""Kernels of the exchange's reduce-only passes in a rocprofv3 kernel trace: each
pass is the run of kernels on one queue from the k_init before a k_xingest to
the next k_mat.  Prints the mean duration of every kernel over those passes,
the mean pass span, and the same for the exchange's own kernels (k_x*).
Usage: python tools/xpass_kernels.py TRACE_DIR
"""
import collections
import csv
import glob
import os
import statistics
import sys


def main():
    d = sys.argv[1]
    f = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    rows = list(csv.DictReader(open(f[0])))
    byq = collections.defaultdict(list)
    for r in rows:
        byq[r.get("Queue_Id", "")].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0]))
    dur = collections.defaultdict(list)
    spans = []
    for q, ev in byq.items():
        ev.sort()
        for i, (s, e, n) in enumerate(ev):
            if n != "k_xingest":
                continue
            j0 = i
            while j0 > 0 and ev[j0][2] != "k_init":
                j0 -= 1
            j1 = i
            while j1 < len(ev) - 1 and ev[j1][2] != "k_mat":
                j1 += 1
            spans.append((ev[j1][1] - ev[j0][0]) / 1e3)
            for s2, e2, n2 in ev[j0:j1 + 1]:
                dur[n2].append((e2 - s2) / 1e3)
    xk = collections.defaultdict(list)
    for r in rows:
        n = r["Kernel_Name"].split("(")[0]
        if n.startswith("k_x") and n != "k_xingest":
            xk[n].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    print("reduce-only passes: %d, mean span %.1f us (k_init .. k_mat, one queue)" % (len(spans), statistics.mean(spans) if spans else 0))
    for n, v in sorted(dur.items(), key=lambda kv: -statistics.mean(kv[1])):
        print("  %-24s %8.1f us  (n=%d)" % (n, statistics.mean(v), len(v)))
    print("exchange kernels:")
    for n, v in sorted(xk.items(), key=lambda kv: -statistics.mean(kv[1])):
        print("  %-24s %8.1f us  (n=%d)" % (n, statistics.mean(v), len(v)))


if __name__ == "__main__":
    main()
