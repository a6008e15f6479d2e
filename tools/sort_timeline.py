"""The last device bytewise sort in a rocprofv3 kernel trace (from its
k_bs_zero / k_bs_init to the end of its k_bs_out2, with the fills and copies
between them): per kernel start, duration and the idle gap before it.
Usage: python tools/sort_timeline.py TRACE_DIR
"""
import csv
import glob
import os
import sys


def main():
    f = glob.glob(os.path.join(sys.argv[1], "**", "*kernel_trace.csv"), recursive=True)
    rows = list(csv.DictReader(open(f[0])))
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0]) for r in rows)
    starts = [i for i, e in enumerate(ev) if e[2] in ("k_bs_zero", "k_bs_init") and (i == 0 or ev[i - 1][2] not in ("k_bs_zero",))]
    if not starts:
        print("no sort found")
        return
    i0 = starts[-1]
    t0, prev, busy = ev[i0][0], ev[i0][0], 0
    for s, e, n in ev[i0:]:
        if not (n.startswith(("k_bs", "k_os", "k_scan", "__amd"))):
            break
        print("%-26s start %8.1f dur %6.1f gap %6.1f" % (n[:26], (s - t0) / 1e3, (e - s) / 1e3, (s - prev) / 1e3))
        busy += e - s
        prev = max(prev, e)
        if n == "k_bs_out2":
            break
    print("span %.1f us, kernels %.1f us" % ((prev - t0) / 1e3, busy / 1e3))


if __name__ == "__main__":
    main()
