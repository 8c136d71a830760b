#!/bin/bash
# Round-end GPU pass (repo root on the GPU box): smoke, GPU parity tests, the
# default bench line, then rocprofv3 stats + PMC passes for mlp512 and gru256.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/re
mkdir -p $O
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
echo "smoke ok"
timeout -k 10 600 python3 -u -m pytest tests/ -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo "gpu tests failed"; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python3 $R/bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
TAG=mlp512 bash $R/tools/profile.sh || exit 1
TAG=gru256 ARGS="--workload go2_gru_256_b4096 --no-cpu --no-latency --no-ctl" bash $R/tools/profile.sh || exit 1
echo "round_end ok"
