#!/bin/bash
# Same-box per-kernel A/B of engine options on one stream (bench.py --serial): a rocprofv3 kernel
# trace of a short bench per option set, then each set's average for the kernels matching a regex.
#   bash flow-q-learning_amd/csrc/tools/ab_serial_opts.sh <regex> "" "dw_stagger=4" ...
set -uo pipefail
RX=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
cd /tmp && export TMPDIR=/tmp
i=0
for spec in "$@"; do
  i=$((i + 1))
  args=()
  IFS=',' read -ra kvs <<< "$spec"
  for kv in "${kvs[@]}"; do [ -n "$kv" ] && args+=(--engine-option "$kv"); done
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/abso_$i" -o run -- \
      python3 "$R/bench.py" --serial --steps 60 --warmup 10 --no-cpu-baseline --kernel-iters 1 --no-probe \
      --preheat-ms 0 --eval-envs 0 --envmodel-train-steps 0 "${args[@]}" > "$O/abso_$i.log" 2>&1 || exit 1
  python3 - "$O/abso_$i/run_kernel_stats.csv" "$RX" "[$spec]" <<'PY'
import csv, re, sys
path, rx, tag = sys.argv[1:4]
tot = 0.0
for row in csv.DictReader(open(path)):
    name = row["Name"]
    if re.search(rx, name):
        tot += float(row["TotalDurationNs"])
        print(f"{tag:16s} {float(row['AverageNs']) / 1000:9.1f} us  x{row['Calls']:>6s}  {name[:80]}")
print(f"{tag:16s} total {tot / 1e3 / 70:9.1f} us per step (70 steps incl. warmup)")
PY
done
