#!/bin/bash
# r05 probes (GPU box, repo root): the two-waves-per-SIMD MFMA/VALU microbenchmark,
# then the in-kernel clock probes (GO2PI_DIAG_CLOCK build) of mlp512, the GRU-256
# tick and the 4096-robot controller tick. Each step under its own time limit.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/probe
mkdir -p $O
if [ -x $R/tools/mfma_2wave.bin ]; then
  timeout -k 10 60 $R/tools/mfma_2wave.bin > $O/mfma_2wave.txt 2>&1 || { echo "mfma_2wave failed"; cat $O/mfma_2wave.txt; exit 1; }
  cat $O/mfma_2wave.txt
fi
[ -n "$NO_CLOCK" ] && exit 0
export GO2PI_LIB=$R/go2_onnx_controller_amd/lib/diag/libgo2pi_clock.so GO2PI_DIAG_STAMPS=1
timeout -k 10 120 python3 $R/tools/clock_probe.py --waves 4 > $O/clock_mlp512.json || exit 1
timeout -k 10 120 python3 $R/tools/clock_probe.py --waves 4 --model go2_gru_256 > $O/clock_gru256.json || exit 1
timeout -k 10 120 python3 $R/tools/clock_probe.py --waves 4 --ctl --model tests/golden/model.onnx > $O/clock_ctl.json || exit 1
echo clocks done
