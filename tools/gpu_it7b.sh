#!/bin/bash
# per-record iteration, then the round-3 profiles part 1
cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash tools/gpu_it7.sh || exit $?
bash tools/gpu_prof_r3a.sh
