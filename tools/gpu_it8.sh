#!/bin/bash
# per-record iteration, then the round-3 profiles part 2 (C3, C4)
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
bash tools/gpu_it7.sh || exit $?
bash tools/profile_round.sh r03 C3 C4
