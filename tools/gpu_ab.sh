#!/bin/bash
# GPU tests T (optional), then each bench A/B line: NAME|ENV|ARGS;NAME|ENV|ARGS...
# (kernel statistics per line under gpurun_out/prof/NAME_*)
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
if [ -n "$T" ]; then
  timeout -k 10 ${TT:-900} python -u -m pytest $T -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/pt_ab.log 2>&1
  rc=$?; tail -3 gpurun_out/pt_ab.log; [ $rc -eq 0 ] || exit $rc
fi
IFS=';' read -ra LINES <<< "$AB"
for l in "${LINES[@]}"; do
  IFS='|' read -r name envs args <<< "$l"
  env $envs bash tools/prof.sh $name $args | grep -v "^W2" | head -9 || exit $?
  grep '^{' gpurun_out/prof/$name.log | python3 -c "
import json,sys
d=json.loads(sys.stdin.read())
out={'value':d['value']}
for k in ('hbm_resident','per_record'):
    if d.get(k): out[k]=d[k]['value']
s=d.get('sql_shape') or {}
for k in ('per_batch','per_record'):
    if k in s: out['sql_'+k]=(s[k]['value'], s[k]['roofline']['avg_launch_ms'], s[k]['lean_batches'], s[k]['replays_onto_record_kernels'])
print('$name', json.dumps(out))"
done
