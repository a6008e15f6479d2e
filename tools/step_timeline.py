"""Timeline of the last engine-group step from a rocprofv3 trace directory:
kernels, memory copies and (if traced) HIP API calls longer than a threshold,
in start order, with the idle gap before each device event.  A step starts at
the last k_init whose pass begins a local pass (the first k_init after a gap
of more than GAP_MS with no kernel), so the exchange pass's k_init is inside
it.
Usage: python tools/step_timeline.py TRACE_DIR [api_min_us=50]
"""
import csv
import glob
import os
import sys

GAP_MS = 2.0


def load(d, pat):
    f = glob.glob(os.path.join(d, "**", pat), recursive=True)
    return list(csv.DictReader(open(f[0]))) if f else []


def main():
    d = sys.argv[1]
    api_min = float(sys.argv[2]) if len(sys.argv) > 2 else 50.0
    ev = []
    for r in load(d, "*kernel_trace.csv"):
        ev.append(("K", r["Kernel_Name"].split("(")[0], int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                   r.get("Queue_Id", "")))
    for r in load(d, "*memory_copy_trace.csv"):
        ev.append(("C", r.get("Direction", "copy") + " " + r.get("Size", r.get("Bytes", "")), int(r["Start_Timestamp"]),
                   int(r["End_Timestamp"]), ""))
    api = [("A", r["Function"], int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r.get("Thread_Id", ""))
           for r in load(d, "*hip_api_trace.csv")]
    ev.sort(key=lambda x: x[2])
    # step starts: a k_init preceded by >= GAP_MS of device idle time
    starts, last_end = [], None
    for i, e in enumerate(ev):
        if e[0] == "K" and e[1].startswith("k_init") and (last_end is None or e[2] - last_end > GAP_MS * 1e6):
            starts.append(i)
        last_end = e[3] if last_end is None else max(last_end, e[3])
    if not starts:
        print("no step found")
        return
    i0 = starts[-2] if len(starts) >= 2 else starts[-1]  # the last full step (the final one may be the untimed call)
    i1 = starts[-1] if len(starts) >= 2 else len(ev)
    seg = ev[i0:i1]
    t0 = seg[0][2]
    tend = max(e[3] for e in seg)
    seg_api = [a for a in api if t0 <= a[2] <= tend and (a[3] - a[2]) / 1e3 >= api_min]
    rows = sorted(seg + seg_api, key=lambda x: x[2])
    prev = t0
    busy = 0
    print("%-2s %-34s %10s %9s %8s" % ("", "event", "start_us", "dur_us", "gap_us"))
    for kind, name, s, e, q in rows:
        gap = (s - prev) / 1e3 if kind != "A" else float("nan")
        print("%-2s %-34s %10.1f %9.1f %8.1f %s" % (kind, name[:34], (s - t0) / 1e3, (e - s) / 1e3, gap, q))
        if kind != "A":
            busy += e - s
            prev = max(prev, e)
    print("step %.1f us, device events %d, summed durations %.1f us" % ((tend - t0) / 1e3, len(seg), busy / 1e3))


if __name__ == "__main__":
    main()
