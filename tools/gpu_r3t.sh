#!/bin/bash
# round 3: LDS-staged k_mvx_extract (tests, C3 chained / per-block, trace) and the C2 k_bd_parse
# lanes A/B (tools/gpu_r3r.sh + tools/gpu_r3s.sh in one call)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
bash tools/gpu_r3r.sh && bash tools/gpu_r3s.sh
