#!/bin/bash
# Round-4 probes in one GPU call: the direct pass-2 table A/B (r04_p2d.sh), then LDS-DMA staging
# on / off, the 8 K SQ counters and the 64 K cf32 PMC traffic (r04_c4b.sh), then the product's
# round evidence (r04_evidence.sh, tag r04e); the large-N front kernel block-width A/B (r04_bw.sh).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-r04n}
bash scripts/r04_p2d.sh $TAG || exit $?
bash scripts/r04_c4b.sh $TAG || exit $?
bash scripts/r04_bw.sh $TAG || exit $?
bash scripts/r04_evidence.sh r04e
