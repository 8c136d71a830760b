#!/bin/bash
# r04 closing pass (GPU box, repo root): GPU parity tests, the batch-1 act() A/B and
# request timeline, then the profile pass (rocprofv3 stats + FETCH/WRITE PMC passes,
# clock probes, default bench line). Summarise with tools/summarize_prof.py --round r04.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out/lat
bash tools/gpu_tests.sh || exit 1
bash tools/r04_latency.sh > gpurun_out/lat/r04_latency.log 2>&1 || { tail -20 gpurun_out/lat/r04_latency.log; exit 1; }
echo latency done
bash tools/r04_profile.sh
