"""Print the kernel timeline of one population step from a rocprofv3
--kernel-trace CSV (developer tool):

  python step_timeline.py <run_kernel_trace.csv> [step_index]

A step is the launches after one finalize_kernel up to the next.  Columns: start offset (us),
duration (us), queue, kernel.  Ends with per-kernel-family busy time and the
step's wall span.
"""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
k = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], r["Queue_Id"]) for r in rows]
k.sort()
# a step's graph ends with finalize_kernel (with the flow prefetch, the next step's sample
# runs inside the previous graph): step = the launches after one finalize up to the next
fin = [i for i, x in enumerate(k) if x[2].startswith("fq::finalize_kernel")]
si = int(sys.argv[2]) if len(sys.argv) > 2 else len(fin) // 2
a, b = fin[si - 1] + 1, fin[si] + 1
t0 = k[a][0]
fam = collections.defaultdict(float)
for s, e, n, q in k[a:b]:
    short = n.replace("void ", "").replace("fq::", "").split("(")[0]
    fam[short] += (e - s) / 1e3
    print(f"{(s - t0) / 1e3:9.1f} {(e - s) / 1e3:8.1f}  q{q}  {short}")
end = max(e for s, e, n, q in k[a:b])
print(f"step span {(end - t0) / 1e3:.1f} us, next step starts at {(k[b][0] - t0) / 1e3:.1f} us" if b < len(k) else
      f"step span {(end - t0) / 1e3:.1f} us")
for n, v in sorted(fam.items(), key=lambda x: -x[1]):
    print(f"{v:9.1f} us  {n}")
print(f"sum of kernel time {sum(fam.values()):.1f} us")
