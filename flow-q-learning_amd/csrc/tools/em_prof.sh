#!/bin/bash
# rocprofv3 kernel stats of the multistep env-model A/B (tools/em_multistep_ab.py), GPU box
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-em}
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_$TAG" -o run -- \
    python3 "$R/flow-q-learning_amd/csrc/tools/em_multistep_ab.py" 10 1 > "$R/gpurun_out/prof_$TAG.log" 2>&1 || exit 1
python3 "$R/flow-q-learning_amd/csrc/tools/prof_summary.py" "$R/gpurun_out/prof_$TAG/run_kernel_stats.csv" 1 | head -12
