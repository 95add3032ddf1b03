#!/bin/bash
# Same-box per-kernel A/B of builds on one stream (bench.py --serial): a rocprofv3 kernel trace of
# a short bench per build, then each build's average for the kernels matching a regex.
#   bash flow-q-learning_amd/csrc/tools/ab_serial.sh <regex> new ref ...   ("new" = the working
#   tree's libfqlpop.so, X = csrc/devlib/libfqlpop_X.so through FQLPOP_LIB)
set -uo pipefail
RX=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
cd /tmp && export TMPDIR=/tmp
for f in "$@"; do
  if [ "$f" = new ]; then unset FQLPOP_LIB; else export FQLPOP_LIB=$R/flow-q-learning_amd/csrc/devlib/libfqlpop_$f.so; fi

  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/abs_$f" -o run -- \
      python3 "$R/bench.py" --diagnostic --serial --steps 60 --warmup 10 --no-cpu-baseline --kernel-iters 1 --no-probe --preheat-ms 0 \
      --eval-envs 0 --envmodel-train-steps 0 > "$O/abs_$f.log" 2>&1 || exit 1
  python3 - "$O/abs_$f/run_kernel_stats.csv" "$RX" "$f" <<'EOF'
import csv, re, sys
path, rx, tag = sys.argv[1:4]
for row in csv.DictReader(open(path)):
    name = row["Name"]
    if re.search(rx, name):
        print(f"{tag:6s} {float(row['AverageNs']) / 1000:9.1f} us  x{row['Calls']:>6s}  {name[:90]}")
EOF
done
