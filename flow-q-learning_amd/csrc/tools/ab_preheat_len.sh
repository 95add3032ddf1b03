#!/bin/bash
# The driver's short command with preheats of different lengths (steps of a throwaway
# population), interleaved; prints value and the sclk / power at the timed region's edges.
#   bash flow-q-learning_amd/csrc/tools/ab_preheat_len.sh "300 1000 2000" [reps]
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
for rep in $(seq 1 ${2:-3}); do
  for ms in $1; do
    timeout -k 5 200 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --eval-envs 0 \
        --envmodel-train-steps 0 --kernel-iters 2 --preheat-ms $ms 2>/dev/null \
      | python -c "import json,sys; d=json.load(sys.stdin); g=d['gpu_clock']; print('[preheat $ms]', d['value'], d['ms_per_step'], d['preheat']['steps'], g['start'].get('sclk_mhz'), g['end'].get('sclk_mhz'), g['start'].get('power_w'), g['end'].get('power_w'))" || exit 1
  done
done
