#!/bin/bash
# one GPU iteration: kernel-variant parity, bench lines, phase split, replay attribution
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
tag=${1:-l}
bash scripts/r02_quick.sh "$tag" && bash scripts/r02_exp.sh "${tag}x"
