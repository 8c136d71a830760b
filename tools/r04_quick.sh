#!/bin/bash
# r04 iteration pass (GPU box, repo root): GPU tests, the batch-1 latency A/B, the clock
# probes (GO2PI_DIAG_CLOCK build) of the controller tick, the GRU-256 tick and mlp512,
# then the default bench line.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out/q
bash $R/tools/gpu_tests.sh || exit 1
bash $R/tools/r04_latency.sh || exit 1
if [ -f $R/go2_onnx_controller_amd/lib/diag/libgo2pi_clock.so ]; then
  export GO2PI_LIB=$R/go2_onnx_controller_amd/lib/diag/libgo2pi_clock.so GO2PI_DIAG_STAMPS=1
  timeout -k 10 120 python3 $R/tools/clock_probe.py --waves 4 --ctl --model tests/golden/model.onnx > $R/gpurun_out/q/clock_ctl.json || exit 1
  timeout -k 10 120 python3 $R/tools/clock_probe.py --waves 4 --model go2_gru_256 > $R/gpurun_out/q/clock_gru256.json || exit 1
  timeout -k 10 120 python3 $R/tools/clock_probe.py --waves 4 > $R/gpurun_out/q/clock_mlp512.json || exit 1
  unset GO2PI_LIB GO2PI_DIAG_STAMPS
  echo clocks done
fi
timeout -k 10 400 python3 $R/bench.py > $R/gpurun_out/q/bench.json 2> $R/gpurun_out/q/bench.err || { echo "bench failed"; tail -20 $R/gpurun_out/q/bench.err; exit 1; }
cat $R/gpurun_out/q/bench.json
