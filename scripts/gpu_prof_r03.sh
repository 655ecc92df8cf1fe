#!/bin/bash
# Round-3 counter evidence: the C5 headline (65536 photo -c -m streams) and C3 (4096 photo -c),
# each as scripts/profile.sh passes (kernel stats, then one PMC group per run).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash scripts/profile.sh r03 --steps 2 --warmup 1 --no-configs || exit $?
bash scripts/profile.sh r03c3 --streams 4096 --no-diff --steps 3 --warmup 1 --no-configs || exit $?
