#!/bin/bash
# Round 3: epilogue woven into the own phase (GO2PI_DIAG_WEAVE) with the own chunk's
# fragment loads front-loaded like w4_chunk's: parity of that build, A/B, clock probes.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/ab3
D=$R/go2_onnx_controller_amd/lib/diag
mkdir -p $O
GO2PI_LIB=$D/libgo2pi_weave.so timeout -k 10 400 python3 -u -m pytest tests/test_gpu_pipeline.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > $O/tests_weave.log 2>&1 || { echo "weave parity failed"; tail -30 $O/tests_weave.log; exit 1; }
tail -1 $O/tests_weave.log
timeout -k 10 600 python3 tools/ab.py --rounds 3 --out $O new weave=weave || exit 1
for v in clock weave_clock; do
  GO2PI_DIAG_STAMPS=1 GO2PI_LIB=$D/libgo2pi_$v.so timeout -k 10 120 python3 tools/clock_probe.py --waves 4 > $O/$v.json 2> $O/$v.err || { echo "$v failed"; exit 1; }
  python3 -c "import json;d=json.load(open('$O/$v.json'));print('$v', d['wg_cycles_median'], round(d['event_us_per_launch'],2), d['phase_cycles_median'], d['pipeline_layer1_subphases'].get('0'))"
done
