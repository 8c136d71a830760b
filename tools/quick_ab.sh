#!/bin/bash
# Quick check of a kernel change on the GPU box: smoke, GPU parity tests, bench lines.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/q
mkdir -p $O
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
echo "smoke ok"
timeout -k 10 600 python3 -u -m pytest tests/ -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo "gpu tests failed"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for wl in go2_mlp_512_b4096 go2_gru_256_b4096; do
  timeout -k 10 120 python3 $R/bench.py --workload $wl --no-cpu --no-latency > $O/b_$wl.json 2> $O/b_$wl.err || { echo "bench $wl failed"; exit 1; }
  python3 -c "import json;d=json.load(open('$O/b_$wl.json'));print('$wl', d['kernel_us'], d['roofline']['frac'], d.get('controller_tick',{}).get('tick_us'))"
done
