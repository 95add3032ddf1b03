#!/bin/bash
# Same-box A/B of runtime switches (developer loop, on the GPU box from the repo root):
#   bash flow-q-learning_amd/csrc/tools/ab_env.sh "ENV=a ENV2=b|--bench-arg" "ENV=c|" ...
# Each argument is "<env assignments>|<extra bench args>"; every config runs twice, interleaved.
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
for rep in 1 2; do
  for spec in "$@"; do
    envs=${spec%%|*}; args=${spec#*|}
    env $envs timeout -k 5 120 python bench.py --diagnostic --steps 400 --no-cpu-baseline --no-probe --eval-envs 0 \
        --envmodel-train-steps 0 $args 2>/dev/null \
      | python -c "import json,sys; d=json.load(sys.stdin); print('[$envs|$args]', d['value'], d['ms_per_step'], d['config']['info_finite'])" || exit 1
  done
done
