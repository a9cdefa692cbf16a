#!/bin/bash
# Round-3 profiles, part 1: C2 and C5 kernel statistics + PMC traffic, C2 per-record statistics + traffic.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
bash tools/profile_round.sh r03 C2 C5 || exit $?
bash tools/prof.sh r03_c2_pr --emit per_record --no-host-input --no-per-record || exit $?
bash tools/traffic.sh c2_pr --emit per_record --no-host-input --no-per-record | tail -3
