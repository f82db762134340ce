#!/bin/bash
# r05 diagnostics in one call: phase stamps, per-workgroup fixed cost, occupancy
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/r05_stamps.sh && bash tools/r05_fixed.sh && bash tools/r05_occ.sh
