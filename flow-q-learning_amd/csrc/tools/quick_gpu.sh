#!/bin/bash
# Developer loop on the GPU box: GPU parity tests, bench, serial kernel profile.
# Usage: bash flow-q-learning_amd/csrc/tools/quick_gpu.sh <tag> [pytest -k expr]
set -uo pipefail
TAG=${1:-q}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
cd "$R"
if [ -n "${2:-}" ]; then K=(-k "$2"); else K=(); fi
timeout -k 10 400 python -m pytest tests -m gpu -x -q "${K[@]}" > "$O/tests_$TAG.log" 2>&1 || { tail -40 "$O/tests_$TAG.log"; exit 1; }
tail -2 "$O/tests_$TAG.log"
timeout -k 10 200 python bench.py --no-cpu-baseline --no-probe --steps 300 > "$O/bench_$TAG.json" 2> "$O/bench_$TAG.err" || exit 1
python -c "import json; d=json.load(open('$O/bench_$TAG.json')); print('bench', d['value'], d['ms_per_step'])"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_$TAG" -o run -- \
    python3 "$R/bench.py" --serial --steps 100 --warmup 20 --no-cpu-baseline --kernel-iters 1 --no-probe --envmodel-train-steps 0 > "$O/prof_$TAG.log" 2>&1 || exit 1
python "$R/flow-q-learning_amd/csrc/tools/prof_summary.py" "$O/prof_$TAG/run_kernel_stats.csv" 120 > "$O/prof_$TAG.txt"; head -16 "$O/prof_$TAG.txt"; true
