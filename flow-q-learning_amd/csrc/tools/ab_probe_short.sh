#!/bin/bash
# The driver's short command (--steps 20 --warmup 5) with the in-step probe on and off,
# interleaved, plus the time each sysfs clock read takes (gpu_clock.*.read_ms).
#   bash flow-q-learning_amd/csrc/tools/ab_probe_short.sh [pairs]
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
for rep in $(seq 1 ${1:-3}); do
  for p in "" "--no-probe"; do
    timeout -k 5 200 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --eval-envs 0 \
        --envmodel-train-steps 0 --kernel-iters 2 $p 2>/dev/null \
      | python -c "import json,sys; d=json.load(sys.stdin); g=d['gpu_clock']; print('[${p:-probe}]', d['value'], d['ms_per_step'], g['start'].get('read_ms'), g['end'].get('read_ms'), g['start'].get('sclk_mhz'), g['end'].get('sclk_mhz'))" || exit 1
  done
done
