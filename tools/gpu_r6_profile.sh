#!/bin/bash
# Round-6 kernel statistics + PMC traffic: the plain C2 pipeline (refreshed)
# and the SQL op shape (per batch, EMIT CHANGES) on C2 and C5.
#   bash tools/gpu_r6_profile.sh [name ...]
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
ARGS="$*"
one() { n=$1; shift; if [ -n "$ARGS" ] && [[ " $ARGS " != *" $n "* ]]; then return 0; fi
  bash tools/prof.sh r06_$n "$@" | grep -v "^W2" || return 1
  bash tools/traffic.sh $n "$@" > /dev/null || return 1
  python3 -c "import json; d=json.load(open('gpurun_out/pmc/traffic_$n.json')); print('$n traffic/batch', d['hbm_bytes_per_batch'], 'batches', d['batches'])"; }
one c2 --config C2 --input hbm --no-hbm --no-per-record --no-sql-shape || exit 1
one c2_sql --config C2 --input hbm --only-sql --sql-emit per_batch --extra-steps 1 || exit 1
one c2_sql_pr --config C2 --input hbm --only-sql --sql-emit per_record --extra-steps 1 || exit 1
one c5_sql --config C5 --input hbm --only-sql --sql-emit per_batch --extra-steps 1 || exit 1
