#!/bin/bash
# rocprofv3 passes over bench.py (run on the GPU box from the repo root):
#   1. kernel trace + stats (per-kernel durations)
#   2. FETCH_SIZE pass, 3. WRITE_SIZE pass (separate --pmc passes, MI355X_MICROARCH.md §rocprofv3)
# Outputs land under gpurun_out/prof_*; tools/summarize_prof.py condenses them into profiles/.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
STEPS=${STEPS:-200}
ARGS=${ARGS:-"--no-cpu --no-latency --no-ctl"}
TAG=${TAG:-mlp}
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_${TAG}_kt -o run -- python3 $R/bench.py --steps $STEPS $ARGS > $R/gpurun_out/prof_${TAG}_kt.log 2>&1 || { echo "kt pass failed rc=$?"; exit 1; }
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $R/gpurun_out/prof_${TAG}_fetch -o run -- python3 $R/bench.py --steps 50 $ARGS > $R/gpurun_out/prof_${TAG}_fetch.log 2>&1 || { echo "fetch pass failed rc=$?"; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $R/gpurun_out/prof_${TAG}_write -o run -- python3 $R/bench.py --steps 50 $ARGS > $R/gpurun_out/prof_${TAG}_write.log 2>&1 || { echo "write pass failed rc=$?"; exit 1; }
echo "profile passes ok"
