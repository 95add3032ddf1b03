"""Per-kernel in-step vs serial times of the population step, for bench.py's roofline block
(every fraction of the BENCH line recomputable from a file under profiles/).

  python kernel_times.py <instep kernel_stats.csv> <steps incl. warmup> <serial pmc table.txt>
                         <serial steps incl. warmup> --commit C --out profiles/kernel_times.json

* in-step: rocprofv3 --kernel-trace --stats of `bench.py --steps S --warmup W --preheat-ms 0
  --kernel-iters 1` (round_profile.sh), every launch of the concurrent step; launches per step
  = round(calls / (S + W)) (the one isolated replay of the dominant kernel is rounded away);
* serial: the `avg us` column of pmc_table.py's table over a `bench.py --serial` run
  (round_pmc.sh), every launch uncontended on one stream.
stretch = in-step average / serial average of the same launch."""
from __future__ import annotations

import argparse
import csv
import datetime
import json
import re


def short(name: str) -> str:
    n = name.replace("void ", "").replace("fq::", "")
    return re.sub(r"\(.*\)$", "", n).strip()


def read_instep(path: str):
    out = {}
    with open(path) as f:
        for row in csv.DictReader(f):
            out[short(row["Name"])] = (int(row["Calls"]), float(row["AverageNs"]) / 1e3)
    return out


def read_serial(path: str):
    out = {}
    with open(path) as f:
        for line in f:
            toks = line.split()
            if len(toks) < 7 or toks[0] == "kernel":
                continue
            try:
                calls, avg = int(toks[-6]), float(toks[-5])
            except ValueError:
                continue
            out[short(" ".join(toks[:-6]))] = (calls, avg)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("instep_csv")
    ap.add_argument("instep_steps", type=int)
    ap.add_argument("serial_table")
    ap.add_argument("serial_steps", type=int)
    ap.add_argument("--commit", required=True)
    ap.add_argument("--out", required=True)
    ap.add_argument("--members", type=int, default=16)
    a = ap.parse_args()
    ins, ser = read_instep(a.instep_csv), read_serial(a.serial_table)
    kern = {}
    for k, (calls, avg) in ins.items():
        per = round(calls / a.instep_steps)
        if per == 0 or k.startswith("__amd") or "rollout" in k or "init_kernel" in k or "emtrain" in k:
            continue
        d = {"launches_per_step": per, "in_step_avg_us": round(avg, 2), "in_step_us_per_step": round(avg * per, 2)}
        if k in ser:
            s_calls, s_avg = ser[k]
            d["serial_avg_us"] = round(s_avg, 2)
            d["serial_us_per_step"] = round(s_avg * round(s_calls / a.serial_steps), 2)
            d["stretch"] = round(avg / s_avg, 3)
        kern[k] = d
    doc = {"commit": a.commit, "date": datetime.date.today().isoformat(), "members": a.members,
           "workload": "cube",
           "instep_source": a.instep_csv, "instep_steps_incl_warmup": a.instep_steps,
           "serial_source": a.serial_table, "serial_steps_incl_warmup": a.serial_steps,
           "kernels": dict(sorted(kern.items(), key=lambda kv: -kv[1]["in_step_us_per_step"]))}
    with open(a.out, "w") as f:
        json.dump(doc, f, indent=1)
    print(json.dumps(doc, indent=1))


if __name__ == "__main__":
    main()
