#!/bin/bash
# The round's rocprofv3 evidence for every bench workload: tools/profile_round.sh per workload (kernel
# trace + stats of the bench command, then separate FETCH/WRITE/SQ/busy --pmc passes), and the dynamic VALU class split
# of the headline (tools/valu_class_pmc.sh). Stops at the first failing step. usage (on the gpurun box):
#   tools/profile_all.sh <tag-prefix>
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
p="$1"
set -o pipefail
tools/profile_round.sh "${p}c3f" &&
tools/profile_round.sh "${p}c3x" --mode exact &&
tools/profile_round.sh "${p}c2f" --config 2 &&
tools/profile_round.sh "${p}c2x" --config 2 --mode exact &&
tools/profile_round.sh "${p}c4f" --config 4 &&
tools/profile_round.sh "${p}c4x" --config 4 --mode exact &&
tools/profile_round.sh "${p}c3ao" --apply-ao &&
tools/valu_class_pmc.sh "${p}c3f" &&
tools/valu_class_pmc.sh "${p}c3x" --mode exact &&
echo "profile_all done"
