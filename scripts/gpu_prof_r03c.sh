#!/bin/bash
# Round-3 counter evidence for the remaining -c -m bench lines (noise 2048, grad 8192, C2 one
# stream), so that every FGK line carries roofline.traffic and issue: stats + PMC passes each.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
export PASSES="stats inst fetch write"
bash scripts/profile.sh r03bn --kind noise --streams 2048 --steps 2 --warmup 1 --no-configs || exit $?
bash scripts/profile.sh r03bg --kind grad --streams 8192 --steps 2 --warmup 1 --no-configs || exit $?
bash scripts/profile.sh r03b1 --streams 1 --steps 2 --warmup 1 --no-configs || exit $?
echo done
