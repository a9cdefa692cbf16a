#!/bin/bash
# round-end validation at HEAD, then the k_seg_apply 512-thread experiment
cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash tools/gpu_r3_end.sh || exit $?
bash tools/gpu_seg512.sh
