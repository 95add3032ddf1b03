"""Per-kernel table from tools/round_pmc.sh's four rocprofv3 passes (developer tool).

Per kernel (averages per dispatch): duration (kernel trace), MFMA-pipe busy fraction =
SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 XCDs x 1024 SIMDs), HBM-side bytes =
2 x FETCH_SIZE + WRITE_SIZE (KiB counters; FETCH_SIZE doubled per MI355X_MICROARCH.md's
gfx950 correction for wide coalesced reads), and the resulting GB/s.

  python pmc_table.py <dir with trace/ mfma/ fetch/ write/> [--json out.json]
"""
import collections
import csv
import glob
import json
import os
import sys


def name(k):
    return k.replace("void ", "").replace("fq::", "").split("(")[0]


def counters(d):
    path = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    disp = collections.defaultdict(lambda: collections.defaultdict(float))
    kn = {}
    for p in path:
        for r in csv.DictReader(open(p)):
            key = r["Dispatch_Id"]
            kn[key] = name(r["Kernel_Name"])
            disp[key][r["Counter_Name"]] += float(r["Counter_Value"])
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for key, c in disp.items():
        for n, v in c.items():
            agg[kn[key]][n].append(v)
    return agg


def main():
    d = sys.argv[1]
    stats = {}
    for p in glob.glob(os.path.join(d, "trace", "**", "*kernel_stats.csv"), recursive=True):
        for r in csv.DictReader(open(p)):
            stats[name(r["Name"])] = (float(r["AverageNs"]) / 1000.0, int(r["Calls"]), float(r["TotalDurationNs"]))
    mf, fe, wr = counters(os.path.join(d, "mfma")), counters(os.path.join(d, "fetch")), counters(os.path.join(d, "write"))
    mean = lambda xs: sum(xs) / len(xs) if xs else float("nan")
    rows = []
    for k, (us, calls, tot) in sorted(stats.items(), key=lambda kv: -kv[1][2]):
        gui = mean(mf.get(k, {}).get("GRBM_GUI_ACTIVE", [])) / 8
        busy = mean(mf.get(k, {}).get("SQ_VALU_MFMA_BUSY_CYCLES", [])) / (gui * 1024) if gui == gui and gui else float("nan")
        fb = 2 * 1024 * mean(fe.get(k, {}).get("FETCH_SIZE", []))
        wb = 1024 * mean(wr.get(k, {}).get("WRITE_SIZE", []))
        rows.append(dict(kernel=k, calls=calls, avg_us=us, mfma_busy=busy, fetch_bytes_x2=fb, write_bytes=wb,
                         hbm_gbs=(fb + wb) / (us * 1e3) if us else float("nan")))
    print(f"{'kernel':58s} {'calls':>5s} {'avg us':>8s} {'mfma':>6s} {'FETCHx2 MB':>10s} {'WRITE MB':>9s} {'GB/s':>7s}")
    for r in rows:
        print(f"{r['kernel'][:58]:58s} {r['calls']:5d} {r['avg_us']:8.1f} {r['mfma_busy']:6.3f} "
              f"{r['fetch_bytes_x2'] / 1e6:10.2f} {r['write_bytes'] / 1e6:9.2f} {r['hbm_gbs']:7.0f}")
    if "--json" in sys.argv:
        with open(sys.argv[sys.argv.index("--json") + 1], "w") as f:
            json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
