#!/bin/bash
# Passes C (config-5 eager A/B, round-1 tree vs HEAD) then B (one-sided lane
# tests, round times, role bench, kernel trace) in one box session.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
bash scripts/r04/gpu_c.sh && bash scripts/r04/gpu_b.sh
