#!/bin/bash
# End-of-round-4 evidence on one box: tools/r04_evidence.sh (GPU suite, smoke, every bench
# workload, cwt / fwt2d traffic, headline rocprofv3 stats) plus FETCH_SIZE / WRITE_SIZE passes
# of the two MODWT benches (headline, cfg5) for profiles/modwt_pmc_traffic.json.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" || exit 2
TAG="${1:-r04final}"
bash tools/r04_evidence.sh "$TAG" || exit $?
PMC_PASSES="1 2" bash tools/pmc.sh "${TAG}_db4" --steps 1 --warmup 1 --no-alt || exit $?
PMC_PASSES="1 2" bash tools/pmc.sh "${TAG}_sym8" --wavelet Symlet8 --levels 6 --steps 1 --warmup 1 --no-alt || exit $?
echo "final evidence done"
