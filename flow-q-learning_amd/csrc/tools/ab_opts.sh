#!/bin/bash
# Same-box A/B of engine options (developer loop, on the GPU box from the repo root):
#   bash flow-q-learning_amd/csrc/tools/ab_opts.sh "dw_stagger=0" "dw_stagger=4" ...
# Each argument is a comma-separated list of NAME=VALUE engine options (empty: defaults);
# every config runs REPS times (default 3), interleaved.  Prints value and ms per step.
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
for rep in $(seq 1 ${REPS:-3}); do
  for spec in "$@"; do
    args=()
    IFS=',' read -ra kvs <<< "$spec"
    for kv in "${kvs[@]}"; do [ -n "$kv" ] && args+=(--engine-option "$kv"); done
    timeout -k 5 120 python bench.py --steps 400 --no-cpu-baseline --no-probe --eval-envs 0 \
        --envmodel-train-steps 0 --kernel-iters 2 "${args[@]}" 2>/dev/null \
      | python -c "import json,sys; d=json.load(sys.stdin); print('[$spec]', d['value'], d['ms_per_step'], d['config']['info_finite'], d['gpu_clock']['start'].get('sclk_mhz'), d['gpu_clock']['end'].get('sclk_mhz'), d['gpu_clock']['end'].get('power_w'))" || exit 1
  done
done
