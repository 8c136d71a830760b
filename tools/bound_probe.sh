#!/bin/bash
# What bounds the batched kernel (GPU box, repo root): GPU tests, the default
# bench line, then the clock probe on the shipped schedule and on its two
# ablations (noload: weight loads replaced by register arithmetic; nomfma: each
# MFMA replaced by one VALU fma). Build first: make -C go2_onnx_controller_amd/csrc diag
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/bound
mkdir -p $O
D=$R/go2_onnx_controller_amd/lib/diag
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 600 python3 -u -m pytest tests/ -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo "gpu tests failed"; tail -30 $O/tests.log; exit 1; }
  tail -2 $O/tests.log
fi
timeout -k 10 300 python3 $R/bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
export GO2PI_DIAG_STAMPS=1
for v in ${VARIANTS:-clock noload_clock nomfma_clock}; do
  for m in ${MODELS:-go2_mlp_512}; do
    GO2PI_LIB=$D/libgo2pi_$v.so timeout -k 10 120 python3 $R/tools/clock_probe.py --model $m > $O/clock_${v}_$m.json 2> $O/clock_${v}_$m.err || { echo "clock $v $m failed"; tail -5 $O/clock_${v}_$m.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/clock_${v}_$m.json'));print('$v $m', d['wg_cycles_median'], d['event_us_per_launch'], d['phase_cycles_median'])"
  done
done
echo "bound_probe ok"
