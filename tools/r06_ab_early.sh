#!/bin/bash
# r06: the pipeline's early flag check (w4_step: the other waves' flags read during the
# own phase, the first LDS-phase operand read before the last own chunk) against base8
# (the build before it): parity of the pipeline paths, A/B on mlp512, GRU-256, LSTM-256,
# shipped and the controller tick, the mlp512 clock probe.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/abearly
mkdir -p $O
D=$R/go2_onnx_controller_amd/lib/diag
timeout -k 10 600 python3 -u -m pytest $R/tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|Timeout" $O/tests.log | head -20; tail -20 $O/tests.log; exit 1; }
tail -n 1 $O/tests.log
timeout -k 10 600 python3 $R/tools/ab.py --rounds 3 --out $O early base8=base8 2>&1 | tee $O/ab_mlp512.txt || exit 1
timeout -k 10 600 python3 $R/tools/ab.py --rounds 2 --workload go2_gru_256_b4096 --out $O early base8=base8 2>&1 | tee $O/ab_gru.txt || exit 1
timeout -k 10 600 python3 $R/tools/ab.py --rounds 2 --workload go2_lstm_256_b4096 --out $O early base8=base8 2>&1 | tee $O/ab_lstm.txt || exit 1
timeout -k 10 600 python3 $R/tools/ab.py --rounds 2 --workload shipped_b4096 --out $O early base8=base8 2>&1 | tee $O/ab_shipped.txt || exit 1
timeout -k 10 600 python3 $R/tools/ab.py --rounds 2 --ctl --workload shipped_b4096 --out $O early base8=base8 2>&1 | tee $O/ab_ctl.txt || exit 1
GO2PI_LIB=$D/libgo2pi_clock.so GO2PI_DIAG_STAMPS=1 timeout -k 10 120 python3 $R/tools/clock_probe.py --waves 4 > $O/clock_mlp512.json || exit 1
python3 -c "import json; d=json.load(open('$O/clock_mlp512.json')); print({k: d[k] for k in ('wg_cycles_median','event_us_per_launch','phase_cycles_median','pipeline_layer1_subphases')})"
