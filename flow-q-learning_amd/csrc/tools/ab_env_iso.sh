#!/bin/bash
# Same-box A/B of runtime switches, printing the step rate AND the dominant kernel's
# isolated launch time (developer loop, on the GPU box from the repo root):
#   bash flow-q-learning_amd/csrc/tools/ab_env_iso.sh "ENV=a|args" "ENV=b|args" ...
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
for rep in 1 2; do
  for spec in "$@"; do
    envs=${spec%%|*}; args=${spec#*|}
    env $envs timeout -k 5 120 python bench.py --diagnostic --steps 400 --no-cpu-baseline --no-probe --eval-envs 0 \
        --envmodel-train-steps 0 --kernel-iters 20 $args 2>/dev/null \
      | python -c "import json,sys; d=json.load(sys.stdin); print('[$envs|$args]', d['value'], d['ms_per_step'], 'iso_us', d['roofline']['isolated_launch_us'])" || exit 1
  done
done
