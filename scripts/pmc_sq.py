"""Mean per-dispatch SQ counters of one kernel from a rocprofv3 --pmc csv.
Usage: python scripts/pmc_sq.py COUNTER_CSV KERNEL_SUBSTR"""
import csv
import sys
from collections import defaultdict

acc = defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    if sys.argv[2] in r["Kernel_Name"]:
        acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k in sorted(acc):
    print(k, sum(acc[k]) / len(acc[k]))
