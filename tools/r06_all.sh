#!/bin/bash
# r06 combined GPU pass: tools/r06_pass.sh (GPU tests, launch probe, clock probes, bench
# lines), then tools/r06_wide.sh's batch-1 act() A/B and request timeline (its tests
# skipped: the full suite ran). A failing step ends the script.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
bash $R/tools/r06_pass.sh || exit 1
SEL_SKIP=1 bash $R/tools/r06_wide.sh || exit 1
