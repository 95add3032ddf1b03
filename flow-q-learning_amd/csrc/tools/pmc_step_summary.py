"""Per-kernel MFMA utilisation and wave-state split of one serial-stream bench
run from a rocprofv3 --pmc counter CSV (developer tool):

  rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY \
      SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE \
      -d out -o run -- python3 bench.py --serial --steps 10 ...
  python pmc_step_summary.py out/run_counter_collection.csv

mfma_busy = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 XCDs x 1024 SIMDs): the
fraction of SIMD-cycles with the matrix pipe busy over the dispatch (cross-check:
the Euler kernel's 0.79 matches its 123 of 155 TF/s measured fp32 MFMA peak).
wait_any / wait_inst / active: SQ_WAIT_ANY, SQ_WAIT_INST_ANY, SQ_ACTIVE_INST_ANY over
SQ_WAVE_CYCLES (wave parked on s_waitcnt/barrier, issue-stalled, issuing).
"""
import collections
import csv
import sys

disp = collections.defaultdict(dict)
for r in csv.DictReader(open(sys.argv[1])):
    k = r["Kernel_Name"].replace("void ", "").replace("fq::", "").split("(")[0]
    key = (k, r["Dispatch_Id"])
    disp[key][r["Counter_Name"]] = disp[key].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
agg = collections.defaultdict(lambda: collections.defaultdict(float))
cnt = collections.Counter()
for (k, _), c in disp.items():
    cnt[k] += 1
    for n, v in c.items():
        agg[k][n] += v
print(f"{'kernel':45s} {'n':>5s} {'us':>8s} {'mfma_busy':>9s} {'wait_any':>8s} {'wait_inst':>9s} {'active':>6s}")
for k in sorted(agg, key=lambda k: -agg[k]["GRBM_GUI_ACTIVE"]):
    a, n = agg[k], cnt[k]
    gui = a["GRBM_GUI_ACTIVE"] / n / 8
    wc = max(a["SQ_WAVE_CYCLES"], 1.0)
    print(f"{k[:45]:45s} {n:5d} {gui / 2.4e3:8.1f} {a['SQ_VALU_MFMA_BUSY_CYCLES'] / n / (gui * 1024):9.3f} "
          f"{a['SQ_WAIT_ANY'] / wc:8.2f} {a['SQ_WAIT_INST_ANY'] / wc:9.2f} {a['SQ_ACTIVE_INST_ANY'] / wc:6.2f}")
