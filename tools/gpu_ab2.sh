#!/bin/bash
# A/B of lean-kernel variants + parity (round 3): compile-time activation, head accumulator chains.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/ab2
mkdir -p $O
timeout -k 10 700 python3 -u -m pytest tests/ -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo "gpu tests failed"; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 600 python3 tools/ab.py --rounds 3 --out $O new rtact,GO2PI_LEAN_RT_ACT=1 head2=head2 prev=head2,GO2PI_LEAN_RT_ACT=1 || exit 1
GO2PI_DIAG_STAMPS=1 GO2PI_LIB=$R/go2_onnx_controller_amd/lib/diag/libgo2pi_clock.so timeout -k 10 120 python3 tools/clock_probe.py --model go2_mlp_512 --waves 4 > $O/clock_mlp512.json 2> $O/clock.err || { echo clock failed; tail $O/clock.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/clock_mlp512.json'));print(d['wg_cycles_median'], d['event_us_per_launch'], d['phase_cycles_median'], d.get('init_subphases'), d.get('pipeline_layer1_subphases'))"
