#!/bin/bash
# One GPU measurement round (run from the repo root on the GPU box):
#   bench (with / without the in-step probe), rocprofv3 kernel trace of the
#   same bench command, and the two PMC passes for the dominant kernel.
# Usage: bash flow-q-learning_amd/csrc/tools/round_profile.sh <tag>
# (the rocprof pass runs without the preheat: its Euler average is then the in-step one,
# as the bench line's roofline.avg_launch_us, plus a single isolated launch)
set -euo pipefail
TAG=${1:-r}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
K=${2:-euler_flow_kernel}   # dominant kernel symbol (fqlpop_dominant_kernel_info)
timeout -k 10 400 python "$R/bench.py" > "$O/bench_$TAG.json" 2> "$O/bench_$TAG.err"
timeout -k 10 300 python "$R/bench.py" --no-probe --no-cpu-baseline > "$O/bench_${TAG}_noprobe.json" 2>> "$O/bench_$TAG.err"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_$TAG" -o run -- \
    python3 "$R/bench.py" --steps 100 --warmup 20 --no-cpu-baseline --kernel-iters 1 --preheat-ms 0 --envmodel-train-steps 0 > "$O/prof_$TAG.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$K" --output-format csv -d "$O/pmcf_$TAG" -o run -- \
    python3 "$R/flow-q-learning_amd/csrc/tools/profile_dominant.py" 20 > "$O/pmcf_$TAG.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$K" --output-format csv -d "$O/pmcw_$TAG" -o run -- \
    python3 "$R/flow-q-learning_amd/csrc/tools/profile_dominant.py" 20 > "$O/pmcw_$TAG.log" 2>&1
echo "round_profile $TAG done"
