#!/bin/bash
# Round 3: GRU policies' dense layers with the compile-time Elu / layer count
# (policy_fused_kernel<..., 1, 3>) vs the previous build (prev): full GPU suite, A/B, clock.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/ab7
D=$R/go2_onnx_controller_amd/lib/diag
mkdir -p $O
timeout -k 10 700 python3 -u -m pytest tests/ -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo "gpu tests failed"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 600 python3 tools/ab.py --rounds 2 --workload go2_gru_256_b4096 --out $O new prev=prev || exit 1
timeout -k 10 600 python3 tools/ab.py --rounds 2 --steps 60 --workload go2_gru_256_b4096_seq100 --out $O new prev=prev || exit 1
GO2PI_DIAG_STAMPS=1 GO2PI_LIB=$D/libgo2pi_clock.so timeout -k 10 120 python3 tools/clock_probe.py --waves 4 --model go2_gru_256 > $O/clock_gru.json 2> $O/clock.err || { echo "clock failed"; exit 1; }
python3 -c "import json;d=json.load(open('$O/clock_gru.json'));print('clock', d['wg_cycles_median'], round(d['event_us_per_launch'],2), d['phase_cycles_median'], d['gru_stage'], d['pipeline_layer1_subphases'].get('0'))"
