#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
HSG_PHASES=1 timeout -k 10 180 python -u tools/dbg/room.py > gpurun_out/dbg_room.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/dbg_room.log | grep -v "hsg phases" | tail -24
exit $rc
