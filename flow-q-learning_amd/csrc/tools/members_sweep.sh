#!/bin/bash
# Per-GPU throughput against the members per GPU (the strong-scaling regime: a P-member
# population over N GPUs runs P/N members per GPU), cube shapes, same box, interleaved.
#   bash flow-q-learning_amd/csrc/tools/members_sweep.sh "1 2 4 8 16" [reps] [extra bench args]
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p "$R/gpurun_out"
for rep in $(seq 1 ${2:-1}); do
  for m in $1; do
    timeout -k 5 150 python bench.py --members $m --steps 300 --warmup 30 --no-cpu-baseline --eval-envs 0 \
        --envmodel-train-steps 0 --kernel-iters 3 ${3:-} 2> "$R/gpurun_out/sweep_m$m.err" \
      | python -c "import json,sys; d=json.load(sys.stdin); print('[members $m]', d['value'], 'member-steps/s', d['ms_per_step'], 'ms/step', 'sclk', d['gpu_clock']['start'].get('sclk_mhz'), 'dominant', d['roofline']['avg_launch_us'], 'us')" || exit 1
  done
done
