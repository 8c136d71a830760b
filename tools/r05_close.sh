#!/bin/bash
# r05 closing pass (GPU box, repo root): GPU tests + batch-1 latency A/B + bench line
# (tools/r05_round.sh), then rocprofv3 stats / PMC passes, clock probes and the full
# bench line (tools/r05_profile.sh).
set -o pipefail
bash tools/r05_round.sh && bash tools/r05_profile.sh
