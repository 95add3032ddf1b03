"""Per-launch HBM traffic of one kernel from rocprofv3 --pmc counter CSVs
(developer tool).  gfx950 corrections (MI355X_MICROARCH.md, HBM section):
FETCH_SIZE (KiB) reports half the bytes of wide coalesced streaming reads, so
it is doubled; WRITE_SIZE (KiB) is taken as is.

  python pmc_summary.py <fetch counter_collection.csv> <write counter_collection.csv> <kernel substring> [out.json]

The JSON records the source commit (FQ_COMMIT in the environment: the box has no .git, so
the caller passes it) and the UTC date of the summary; bench.py copies both into the
roofline's traffic_source.
"""
import csv
import datetime
import json
import os
import sys


def per_dispatch(path, counter, needle):
    vals = {}
    for r in csv.DictReader(open(path)):
        if needle in r.get("Kernel_Name", "") and r.get("Counter_Name") == counter:
            vals[r["Dispatch_Id"]] = vals.get(r["Dispatch_Id"], 0.0) + float(r["Counter_Value"])
    return list(vals.values())


fetch = per_dispatch(sys.argv[1], "FETCH_SIZE", sys.argv[3])
write = per_dispatch(sys.argv[2], "WRITE_SIZE", sys.argv[3])
f = sum(fetch) / max(1, len(fetch)) * 1024
w = sum(write) / max(1, len(write)) * 1024
print(f"dispatches: fetch {len(fetch)}, write {len(write)}")
print(f"FETCH_SIZE raw {f / 1e6:.3f} MB/launch -> corrected x2 {2 * f / 1e6:.3f} MB")
print(f"WRITE_SIZE {w / 1e6:.3f} MB/launch")
print(f"traffic (corrected) {(2 * f + w) / 1e6:.3f} MB/launch")

if len(sys.argv) > 4:
    with open(sys.argv[4], "w") as fo:
        json.dump({"kernel_regex": sys.argv[3], "members": int(os.environ.get("FQ_MEMBERS", "16")),
                   "workload": os.environ.get("FQ_WORKLOAD", "cube"), "dispatches": len(fetch),
                   "commit": os.environ.get("FQ_COMMIT"),
                   "date": datetime.datetime.now(datetime.timezone.utc).strftime("%Y-%m-%dT%H:%M:%SZ"),
                   "fetch_size_bytes_raw": f, "fetch_bytes_corrected_x2": 2 * f, "write_bytes": w,
                   "traffic_bytes_per_launch": 2 * f + w,
                   "note": "FETCH_SIZE doubled per MI355X_MICROARCH.md (gfx950 counts 64 B per 128 B request); "
                           "WRITE_SIZE as is (4-B-per-lane epilogue stores: uncalibrated width)"}, fo, indent=1)
