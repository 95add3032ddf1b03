#!/bin/bash
# Concurrent-step kernel timeline on the GPU box (developer loop):
#   bash flow-q-learning_amd/csrc/tools/timeline_gpu.sh <tag> [extra bench args, e.g. --members 2]
set -uo pipefail
TAG=${1:-t}
shift || true
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$O/tl_$TAG" -o run -- \
    python3 "$R/bench.py" --diagnostic --steps 60 --warmup 20 --no-cpu-baseline --kernel-iters 1 --no-probe --eval-envs 0 \
    --envmodel-train-steps 0 "$@" > "$O/tl_$TAG.log" 2>&1 || exit 1
python3 "$R/flow-q-learning_amd/csrc/tools/step_timeline.py" "$O/tl_$TAG/run_kernel_trace.csv" > "$O/tl_$TAG.txt"
cat "$O/tl_$TAG.txt"
