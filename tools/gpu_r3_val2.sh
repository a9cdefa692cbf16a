#!/bin/bash
# the k_seg_apply 512-thread comparison, then the round-end validation at HEAD
cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash tools/gpu_seg512.sh || exit $?
bash tools/gpu_r3_end.sh
