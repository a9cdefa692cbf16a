#!/bin/bash
# table-room sizing: lean / window parity tests, C2 and C5 lines; per-record bucket sizes
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/prof; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_lean.py -x -v --timeout 200 --timeout-method thread > gpurun_out/pt_it10a.log 2>&1; rc=$?
tail -12 gpurun_out/pt_it10a.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
  -k "tumbling or hopping or lean or messy or configs or per_record or segments or retention or spill or grow" > gpurun_out/pt_it10b.log 2>&1; rc=$?
tail -3 gpurun_out/pt_it10b.log; [ $rc -eq 0 ] || exit $rc
for c in C2 C5 C3; do
  timeout -k 10 300 python bench.py --config $c --steps 3 --warmup 1 --cpu-seconds 0 --no-host-input --no-per-record > gpurun_out/b_it10_$c.log 2>&1 || { tail -20 gpurun_out/b_it10_$c.log; exit 1; }
  echo "$c $(tail -1 gpurun_out/b_it10_$c.log | cut -c1-110)"
done
for B in 1024 4096 8192; do
  HSG_PR_BUCKET_RECS=$B timeout -k 10 300 python bench.py --emit per_record --steps 3 --warmup 1 --cpu-seconds 0 --no-host-input --no-per-record > gpurun_out/b_pr_$B.log 2>&1 || { tail -20 gpurun_out/b_pr_$B.log; exit 1; }
  echo "B=$B $(tail -1 gpurun_out/b_pr_$B.log | cut -c1-110)"
done
