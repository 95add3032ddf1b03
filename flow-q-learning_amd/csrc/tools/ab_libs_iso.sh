#!/bin/bash
# Same-box A/B of builds with the dominant kernel's isolated launch time (developer loop):
#   bash flow-q-learning_amd/csrc/tools/ab_libs_iso.sh new ref ...   (as ab_libs.sh)
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
for rep in 1 2; do
  for f in "$@"; do
    if [ "$f" = new ]; then unset FQLPOP_LIB; else export FQLPOP_LIB=$R/flow-q-learning_amd/csrc/devlib/libfqlpop_$f.so; fi
    timeout -k 5 120 python bench.py --diagnostic --steps 400 --no-cpu-baseline --no-probe --eval-envs 0 --envmodel-train-steps 0 \
        --kernel-iters 50 2>/dev/null \
      | python -c "import json,sys; d=json.load(sys.stdin); print('$f', d['value'], d['ms_per_step'], 'iso_us', d['roofline']['isolated_launch_us'])" || exit 1
  done
done
