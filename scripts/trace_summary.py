"""Per-kernel duration distribution from a rocprofv3 --kernel-trace CSV
(kernel_trace.csv), for the kernels whose name contains KERNEL_SUBSTR:
dispatches, mean, median, p10, p90, min (µs).  The --stats mean is inflated
by a few long dispatches the tracer itself delays; the median is the figure
to set beside bench.py's per-launch time from HIP events.
Usage: python scripts/trace_summary.py KERNEL_TRACE_CSV KERNEL_SUBSTR [OUT_JSON]"""
import csv
import json
import sys

import numpy as np

path, kern = sys.argv[1], sys.argv[2]
d = np.array([(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
              for r in csv.DictReader(open(path)) if kern in r["Kernel_Name"]])
rec = {"kernel": kern, "dispatches": int(d.size), "mean_us": round(float(d.mean()), 3),
       "median_us": round(float(np.median(d)), 3), "p10_us": round(float(np.percentile(d, 10)), 3),
       "p90_us": round(float(np.percentile(d, 90)), 3), "min_us": round(float(d.min()), 3)}
print(json.dumps(rec))
if len(sys.argv) > 3:
    json.dump(rec, open(sys.argv[3], "w"), indent=1)
