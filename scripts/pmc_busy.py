"""Per-dispatch busy time of one kernel from a rocprofv3 --pmc pass of
GRBM_GUI_ACTIVE (and SQ_BUSY_CYCLES), converted to microseconds with the
shader clock the kernel ran at.

GRBM_GUI_ACTIVE counts the cycles the graphics block was busy during the
dispatch, summed over the 8 XCDs (MI355X_MICROARCH.md, DVFS give-back: the
effective clock is GRBM_GUI_ACTIVE / 8 / wall), so busy_us = GRBM_GUI_ACTIVE
/ 8 / f_clk.  f_clk comes from the roofline record of the same command
(bench.py --record: the span build's delta(s_memtime) / delta(s_memrealtime)
x 100 MHz, median over waves).
Usage: python scripts/pmc_busy.py COUNTER_CSV KERNEL_SUBSTR RECORD_JSON OUT_JSON"""
import csv
import json
import sys

import numpy as np


def per_dispatch(path, kernel, name):
    v = {}
    for r in csv.DictReader(open(path)):
        if kernel in r["Kernel_Name"] and r["Counter_Name"] == name:
            d = r.get("Dispatch_Id") or r.get("Correlation_Id") or str(len(v))
            v[d] = v.get(d, 0.0) + float(r["Counter_Value"])
    return np.array(list(v.values()), np.float64)


def main():
    path, kernel, record, out = sys.argv[1:5]
    rec = json.load(open(record))
    clk = float(rec["span"]["shader_clock_mhz_median"])
    g = per_dispatch(path, kernel, "GRBM_GUI_ACTIVE")
    sq = per_dispatch(path, kernel, "SQ_BUSY_CYCLES")
    busy = g / 8.0 / clk  # us
    bpl = rec["bytes_per_launch"]
    res = {"kernel": kernel, "dispatches": int(len(g)), "shader_clock_mhz": clk, "clock_source": record,
           "GRBM_GUI_ACTIVE_mean": float(g.mean()), "SQ_BUSY_CYCLES_mean": float(sq.mean()) if len(sq) else None,
           "busy_us_mean": round(float(busy.mean()), 4), "busy_us_median": round(float(np.median(busy)), 4),
           "busy_us_p10_p90": [round(float(np.percentile(busy, 10)), 4), round(float(np.percentile(busy, 90)), 4)],
           "ms_per_step_of_the_record": rec["ms_per_step"],
           "frac_busy": round(bpl / (float(np.median(busy)) * 1e-6) / 1e9 / rec["peak_GBs"], 4),
           "how": "busy_us = GRBM_GUI_ACTIVE / 8 XCDs / shader clock (MHz); the counter pass is its own rocprofv3 "
                  "--pmc run of the record's command (counters serialise the dispatches, so busy_us is one "
                  "dispatch's own busy time, not the per-step period)"}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
