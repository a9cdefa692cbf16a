#!/bin/bash
# One build -> measure iteration on the GPU box:
#   T="tests/a.py tests/b.py" B="bench args|bench args" bash tools/gpu_step.sh
# runs the named GPU tests (one pytest process), then each bench line; stops at
# the first failure (GPU faults, aborts and timeouts included).
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
if [ -n "$T" ]; then
  timeout -k 10 ${TT:-900} python -u -m pytest $T -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pt.log 2>&1
  rc=$?; grep -E "PASSED|FAILED|ERROR" gpurun_out/pt.log | grep -v PASSED | head -20; tail -3 gpurun_out/pt.log
  [ $rc -eq 0 ] || exit $rc
fi
i=0
IFS='|' read -ra BL <<< "$B"
for a in "${BL[@]}"; do
  i=$((i + 1))
  timeout -k 10 600 python bench.py $a > gpurun_out/b$i.log 2>&1
  rc=$?; echo "== bench $a rc=$rc"; tail -1 gpurun_out/b$i.log | cut -c1-2500
  [ $rc -eq 0 ] || { tail -20 gpurun_out/b$i.log; exit $rc; }
done
