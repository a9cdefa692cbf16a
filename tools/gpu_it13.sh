#!/bin/bash
# table-room sizing: debug stream, every GPU test, default bench line, C5 / C3 / C4 lines
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 180 python -u tools/dbg/room.py > gpurun_out/dbg_room.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/dbg_room.log | tail -14; [ $rc -eq 0 ] || exit $rc
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pt_it13.log 2>&1; rc=$?
tail -4 gpurun_out/pt_it13.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > gpurun_out/b_it13_default.log 2>&1 || { tail -20 gpurun_out/b_it13_default.log; exit 1; }
tail -1 gpurun_out/b_it13_default.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('default', d['value'], d['table_slots'], d['host_input'] and d['host_input'].get('value'), d['per_record'] and d['per_record'].get('value'))"
for c in C5 C3 C4; do
  timeout -k 10 300 python bench.py --config $c --steps 2 --warmup 1 --cpu-seconds 0 --no-host-input --no-per-record > gpurun_out/b_it13_$c.log 2>&1 || { tail -20 gpurun_out/b_it13_$c.log; exit 1; }
  tail -1 gpurun_out/b_it13_$c.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$c', d['value'], d['table_slots'], d['table_grow_events'])"
done
bash tools/prof.sh it_c2pr13 --emit per_record --no-host-input --no-per-record
