"""k_map durations of every pass in a rocprofv3 kernel trace (TRACE_DIR), and
their mean / min / max: the spread between passes of the async bench."""
import csv
import glob
import os
import statistics
import sys

f = glob.glob(os.path.join(sys.argv[1], "**", "*kernel_trace.csv"), recursive=True)[0]
d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in csv.DictReader(open(f))
     if r["Kernel_Name"].startswith("k_map")]
print("k_map us per pass:", " ".join("%.0f" % x for x in d))
print("mean %.1f  min %.1f  max %.1f  (n=%d)" % (statistics.mean(d), min(d), max(d), len(d)))
