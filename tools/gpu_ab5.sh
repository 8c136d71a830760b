#!/bin/bash
# Round 3: lean Elu kernel with the bias in the accumulator and a packed epilogue vs the
# previous build (nhc): parity, A/B, clock probe.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/ab5
D=$R/go2_onnx_controller_amd/lib/diag
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_pipeline.py tests/test_gpu_parity.py tests/test_gpu_boundary.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo "parity failed"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 600 python3 tools/ab.py --rounds 3 --out $O new nhc=nhc || exit 1
timeout -k 10 600 python3 tools/ab.py --rounds 2 --workload shipped_b4096 --out $O new nhc=nhc || exit 1
GO2PI_DIAG_STAMPS=1 GO2PI_LIB=$D/libgo2pi_clock.so timeout -k 10 120 python3 tools/clock_probe.py --waves 4 > $O/clock.json 2> $O/clock.err || { echo "clock failed"; exit 1; }
python3 -c "import json;d=json.load(open('$O/clock.json'));print('clock', d['wg_cycles_median'], round(d['event_us_per_launch'],2), d['phase_cycles_median'], d['pipeline_layer1_subphases'].get('0'))"
