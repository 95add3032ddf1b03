#!/bin/bash
# Same-box A/B of the HIP runtime's hardware-queue count per process (GPU_MAX_HW_QUEUES,
# default 4 on the box): the default bench step, interleaved.
#   bash flow-q-learning_amd/csrc/tools/ab_hwq.sh "4 8 16" [reps]
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
for rep in $(seq 1 ${2:-3}); do
  for q in $1; do
    GPU_MAX_HW_QUEUES=$q timeout -k 5 120 python bench.py --steps 400 --no-cpu-baseline --no-probe --eval-envs 0 \
        --envmodel-train-steps 0 --kernel-iters 2 2>/dev/null \
      | python -c "import json,sys; d=json.load(sys.stdin); print('[hwq $q]', d['value'], d['ms_per_step'], d['gpu_clock']['start'].get('sclk_mhz'), d['gpu_clock']['end'].get('power_w'))" || exit 1
  done
done
