#!/bin/bash
# Same-box per-kernel A/B of developer library builds (FQLPOP_LIB, bench.py --diagnostic):
#   OPTS="dw_tile_critic=14" bash flow-q-learning_amd/csrc/tools/ab_serial_libs.sh <regex> <lib.so> ...
set -uo pipefail
RX=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
cd /tmp && export TMPDIR=/tmp
args=()
IFS=',' read -ra kvs <<< "${OPTS:-}"
for kv in "${kvs[@]}"; do [ -n "$kv" ] && args+=(--engine-option "$kv"); done
i=0
for lib in "$@"; do
  i=$((i + 1))
  export FQLPOP_LIB=$R/$lib
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/abl_$i" -o run -- \
      python3 "$R/bench.py" --serial --diagnostic --steps 60 --warmup 10 --no-cpu-baseline --kernel-iters 1 \
      --no-probe --preheat-ms 0 --eval-envs 0 --envmodel-train-steps 0 "${args[@]}" > "$O/abl_$i.log" 2>&1 || exit 1
  python3 - "$O/abl_$i/run_kernel_stats.csv" "$RX" "[$(basename $lib)]" <<'PY'
import csv, re, sys
path, rx, tag = sys.argv[1:4]
for row in csv.DictReader(open(path)):
    if re.search(rx, row["Name"]):
        print(f"{tag:24s} {float(row['AverageNs']) / 1000:9.1f} us  x{row['Calls']:>6s}  {row['Name'][:70]}")
PY
done
