#!/bin/bash
# Same-box A/B of engine options (developer loop, on the GPU box from the repo root):
#   [REPS=3] [BENCH_ARGS="--members 2"] bash flow-q-learning_amd/csrc/tools/ab_opts.sh "" "split=0" ...
# Each argument is a comma-separated list of NAME=VALUE engine options (empty: defaults) or
# bench flags (items starting with --, e.g. "--no-graph"); every config runs REPS times,
# interleaved.  Prints value and ms per step (PROBE=1: with the in-step probe, and the dominant
# launch's in-step duration).
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
for rep in $(seq 1 ${REPS:-3}); do
  for spec in "$@"; do
    args=()
    IFS=',' read -ra kvs <<< "$spec"
    for kv in "${kvs[@]}"; do
      case "$kv" in
        --*) args+=("$kv") ;;
        "") ;;
        *) args+=(--engine-option "$kv") ;;
      esac
    done
    probe=--no-probe
    [ "${PROBE:-0}" = 1 ] && probe=
    timeout -k 5 120 python bench.py --steps ${STEPS:-400} --no-cpu-baseline $probe --eval-envs 0 \
        --envmodel-train-steps 0 --kernel-iters 2 ${BENCH_ARGS:-} "${args[@]}" 2>/dev/null \
      | python -c "import json,sys; d=json.load(sys.stdin); print('[$spec]', d['value'], d['ms_per_step'], d['config']['info_finite'], d['gpu_clock']['start'].get('sclk_mhz'), d['gpu_clock']['end'].get('sclk_mhz'), d['gpu_clock']['end'].get('power_w'), 'dominant_us', d['roofline']['avg_launch_us'] if d['roofline']['launches_timed'] else None)" || exit 1
  done
done
