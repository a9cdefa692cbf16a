#!/bin/bash
# half-tile staged scatter: partition/lean parity, C2 / C5 lines, C2 kernel statistics
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/prof; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
  -k "lean or configs or tumbling or part or messy or exchange or unwindowed or per_record or PER_RECORD or segments or changes" > gpurun_out/pt_it14.log 2>&1; rc=$?
tail -2 gpurun_out/pt_it14.log; [ $rc -eq 0 ] || exit $rc
for c in C2 C5; do
  timeout -k 10 300 python bench.py --config $c --steps 5 --warmup 1 --cpu-seconds 0 --no-host-input --no-per-record > gpurun_out/b_it14_$c.log 2>&1 || { tail -20 gpurun_out/b_it14_$c.log; exit 1; }
  tail -1 gpurun_out/b_it14_$c.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$c', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'])"
done
bash tools/prof.sh it_c2_14 --no-host-input --no-per-record
timeout -k 10 300 python bench.py --emit per_record --steps 3 --warmup 1 --cpu-seconds 0 --no-host-input --no-per-record > gpurun_out/b_it14_pr.log 2>&1 || { tail -20 gpurun_out/b_it14_pr.log; exit 1; }
tail -1 gpurun_out/b_it14_pr.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('C2 per-record', d['value'], d['ms_per_step'])"
bash tools/prof.sh it_c2pr14 --emit per_record --no-host-input --no-per-record
