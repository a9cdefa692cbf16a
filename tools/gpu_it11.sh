#!/bin/bash
# debug the table-room holds; per-record bucket sizes
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 180 python -u tools/dbg/room.py > gpurun_out/dbg_room.log 2>&1; rc=$?
cat gpurun_out/dbg_room.log | grep -v amdgpu.ids | tail -20
case $rc in 0|1) ;; *) echo "room.py rc=$rc"; exit $rc;; esac
for B in 1024 4096 8192; do
  HSG_PR_BUCKET_RECS=$B timeout -k 10 300 python bench.py --emit per_record --steps 3 --warmup 1 --cpu-seconds 0 --no-host-input --no-per-record > gpurun_out/b_pr_$B.log 2>&1 || { tail -20 gpurun_out/b_pr_$B.log; exit 1; }
  echo "B=$B $(tail -1 gpurun_out/b_pr_$B.log | cut -c1-110)"
done
