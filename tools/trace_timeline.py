"""Timeline of one pass from a rocprofv3 kernel trace: per kernel start offset,
duration and the idle gap before it.  A pass starts at each k_init launch.
Usage: python tools/trace_timeline.py TRACE_DIR [pass_index=-1]
"""
import csv
import glob
import os
import sys


def main():
    d = sys.argv[1]
    idx = int(sys.argv[2]) if len(sys.argv) > 2 else -1
    f = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)[0]
    rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
    passes, cur = [], None
    for r in rows:
        name = r["Kernel_Name"].split("(")[0]
        if name.startswith("k_init"):
            cur = []
            passes.append(cur)
        if cur is not None and name.startswith("k_"):
            cur.append((name, int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    p = passes[idx]
    t0, prev = p[0][1], p[0][1]
    busy = 0
    print("%-22s %9s %9s %8s" % ("kernel", "start_us", "dur_us", "gap_us"))
    for name, s, e in p:
        print("%-22s %9.1f %9.1f %8.1f" % (name, (s - t0) / 1e3, (e - s) / 1e3, (s - prev) / 1e3))
        busy += e - s
        prev = e
    print("pass %.1f us, kernels busy %.1f us, idle %.1f us, %d launches"
          % ((prev - t0) / 1e3, busy / 1e3, (prev - t0 - busy) / 1e3, len(p)))


if __name__ == "__main__":
    main()
