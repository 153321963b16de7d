#!/bin/bash
# round 3: rocprof stats + PMC passes at the final code (tools/profile_round.sh)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
PROF_OUT=gpurun_out/r3zl/prof bash tools/profile_round.sh || { echo profile failed; exit 1; }
echo done
