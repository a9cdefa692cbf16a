#!/bin/bash
# per-record: parity tests, then the C2 per-record line at three bucket sizes
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/prof; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
  -k "per_record or PER_RECORD or segments or messy or emit_changes or changes" > gpurun_out/pt_it9.log 2>&1; rc=$?
tail -2 gpurun_out/pt_it9.log; [ $rc -eq 0 ] || exit $rc
for B in 1024 4096 8192; do
  HSG_PR_BUCKET_RECS=$B timeout -k 10 300 python bench.py --emit per_record --steps 3 --warmup 1 --cpu-seconds 0 --no-host-input --no-per-record > gpurun_out/b_pr_$B.log 2>&1 || { tail -20 gpurun_out/b_pr_$B.log; exit 1; }
  echo "B=$B $(tail -1 gpurun_out/b_pr_$B.log | cut -c1-120)"
done
HSG_PR_BUCKET_RECS=${BEST:-8192} bash tools/prof.sh it_c2pr9 --emit per_record --no-host-input --no-per-record
