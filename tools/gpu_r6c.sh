#!/bin/bash
# Round-6 session C: session A (suite, default / extended / RE2 lines, SQ
# counters) then session B (hit-slice A/B, wave timeline).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/gpu_r6a.sh ${1:-r6a2} && bash tools/gpu_r6b.sh ${2:-r6b}
