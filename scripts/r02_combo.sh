#!/bin/bash
# planner + scratch parity, C4 line, then the quick loop (wide-kernel parity, C3/C2 lines, C3 phases)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
tag=${1:-cb}
bash scripts/r02_plan.sh "${tag}p" || exit $?
bash scripts/r02_quick.sh "${tag}q" || exit $?
bash scripts/r02_phase.sh "${tag}h"
