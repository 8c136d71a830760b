#!/bin/bash
# GPU parity tests only (repo root on the GPU box); optional pytest selection in $SEL.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/t
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests/ -m gpu -x -v --timeout 120 --timeout-method thread ${SEL:-} > $O/tests.log 2>&1 || { echo "gpu tests failed"; grep -E "PASSED|FAILED|ERROR" $O/tests.log | tail -5; tail -60 $O/tests.log; exit 1; }
tail -2 $O/tests.log
