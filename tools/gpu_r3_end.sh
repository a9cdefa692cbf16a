#!/bin/bash
# Round-3 end: every GPU test, smoke, the default bench line, C2 kernel statistics + traffic,
# per-record statistics + traffic, the force-exchange line.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/prof gpurun_out/pmc; export TMPDIR=/tmp
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pt_end.log 2>&1; rc=$?
tail -3 gpurun_out/pt_end.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_end.log 2>&1 || { tail -5 gpurun_out/smoke_end.log; exit 1; }
tail -1 gpurun_out/smoke_end.log
timeout -k 10 300 python bench.py > gpurun_out/b_end_default.log 2>&1 || { tail -20 gpurun_out/b_end_default.log; exit 1; }
tail -1 gpurun_out/b_end_default.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('default', d['value'], d['table_slots'], d['roofline']['traffic'], d['host_input']['value'], d['per_record']['value'])"
bash tools/prof.sh r03_end_c2 --no-host-input --no-per-record || exit $?
bash tools/traffic.sh c2 --config C2 --no-host-input --no-per-record | tail -2
bash tools/traffic.sh c2_pr --emit per_record --no-host-input --no-per-record | tail -2
timeout -k 10 300 python bench.py --force-exchange --steps 3 --warmup 1 --cpu-seconds 0 --no-host-input --no-per-record > gpurun_out/b_end_fx.log 2>&1 || { tail -20 gpurun_out/b_end_fx.log; exit 1; }
tail -1 gpurun_out/b_end_fx.log | cut -c1-120
