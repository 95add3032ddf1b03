"""Offline analysis of a FQLPOP_PHASE_DUMP file (critic backward): which blocks shared a CU,
and in what order they started.  python placement.py <dump> [stride=48]"""
import collections
import sys

import numpy as np

st = int(sys.argv[2]) if len(sys.argv) > 2 else 48
a = np.fromfile(sys.argv[1], dtype=np.uint64).reshape(-1, st)
start, end = a[:, 0].astype(np.int64), a[:, 1].astype(np.int64)
hw, xcc = a[:, st - 1].astype(np.int64), a[:, st - 2].astype(np.int64)
t0 = start.min()
cu = collections.defaultdict(list)
for b in range(a.shape[0]):
    key = (int(xcc[b]) & 0xF, (int(hw[b]) >> 8) & 0xFF)
    cu[key].append((int(start[b] - t0), int(end[b] - t0), b))
print("blocks", a.shape[0], "CUs", len(cu), "blocks per CU", collections.Counter(len(v) for v in cu.values()))
diffs = collections.Counter()
overlap_pairs = 0
for key, v in sorted(cu.items())[:6]:
    v.sort()
    print(key, [(s // 100, e // 100, b) for s, e, b in v])  # us
for v in cu.values():
    v.sort()
    if len(v) >= 2:
        diffs[v[1][2] - v[0][2]] += 1
print("blockIdx difference of the first two blocks on a CU:", diffs.most_common(8))
