#!/bin/bash
# the k_seg_apply 512-thread comparison, then smoke and the default bench line at HEAD
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
bash tools/gpu_seg512.sh || exit $?
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_end.log 2>&1 || { tail -5 gpurun_out/smoke_end.log; exit 1; }
tail -1 gpurun_out/smoke_end.log
timeout -k 10 300 python bench.py > gpurun_out/b_end_default.log 2>&1 || { tail -20 gpurun_out/b_end_default.log; exit 1; }
tail -1 gpurun_out/b_end_default.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('default', d['value'], d['table_slots'], d['host_input']['value'], d['per_record']['value'])"
