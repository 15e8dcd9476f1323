#!/bin/bash
# round 6 final tree (MFMA stem, multi-row resize), part 2: the profile set (tools/profile_set.sh):
# default line, traced bench, profile-only kernel trace, PMC traffic and
# stall passes, then the default line again with the traffic in place
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash tools/profile_set.sh r06an || exit 1
echo done
