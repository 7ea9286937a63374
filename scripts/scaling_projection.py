"""Assemble the 1 -> 8 GPU projection from per-shard bench lines measured on
ONE GPU.  Each rank of an N-GPU run steps its own shard
with no collective on the data path, so the N-GPU rate is N x the
one-GPU rate at the per-GPU batch:
  weak   (65 536 envs per GPU, the headline): N x rate(65 536)
  strong (65 536 envs in total):              N x rate(65 536 / N)
Both forms of the bench command are used: the driver's 20-step form and the
1 000-step default.  A PROJECTION from one-GPU measurements, not a multi-GPU
measurement.
Usage: python scripts/scaling_projection.py OUT_JSON LINE_FILE..."""
import json
import sys


def main():
    out, files = sys.argv[1], sys.argv[2:]
    rates = {}
    for f in files:
        line = [x for x in open(f) if x.startswith("{")][-1]
        d = json.loads(line)
        form = "driver_form_20_steps" if d["steps"] == 20 else f"{d['steps']}_steps"
        rates.setdefault(form, {})[d["config"]["batch_per_gpu"]] = {"value": d["value"], "ms_per_step": d["ms_per_step"],
                                                                    "file": f}
    proj = {}
    for form, r in rates.items():
        full = r.get(65536)
        p = {"weak": {}, "strong": {}}
        for n in (1, 2, 4, 8):
            if full:
                p["weak"][n] = {"per_gpu_batch": 65536, "value": round(n * full["value"], 1), "efficiency": 1.0}
            b = 65536 // n
            if b in r and full:
                v = n * r[b]["value"]
                p["strong"][n] = {"per_gpu_batch": b, "value": round(v, 1),
                                  "efficiency": round(v / (n * full["value"]), 3)}
        proj[form] = {"per_shard": r, "projection": p}
    res = {"what": "1 -> 8 GPU projection from one-GPU per-shard measurements (no collective on the data path); "
                   "NOT a multi-GPU measurement: no 8-GPU node was available to this session",
           "forms": proj}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
