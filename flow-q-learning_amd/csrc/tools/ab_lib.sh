#!/bin/bash
# Same-box A/B of two builds (developer loop, on the GPU box from the repo root):
#   make -C flow-q-learning_amd/csrc OUT=devlib/libfqlpop_ref.so   # the reference build, here
#   bash flow-q-learning_amd/csrc/tools/ab_lib.sh [extra bench args]
# alternates the working-tree library and libfqlpop_ref.so (FQLPOP_LIB) three times each.
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
for f in new ref new ref new ref; do
    if [ $f = ref ]; then export FQLPOP_LIB=$R/flow-q-learning_amd/csrc/devlib/libfqlpop_ref.so; else unset FQLPOP_LIB; fi
    timeout -k 5 120 python bench.py --diagnostic --steps 400 --no-cpu-baseline --no-probe --eval-envs 0 --envmodel-train-steps 0 "$@" \
        2>/dev/null | python -c "import json,sys; d=json.load(sys.stdin); print('$f', d['value'], d['ms_per_step'])" || exit 1
done
