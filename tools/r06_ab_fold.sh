#!/bin/bash
# r06: the GPU test suite on the current default build, then A/B of the default (log2(e)
# folded into the pipeline weights) against avt (the previous default) for mlp512, GRU,
# LSTM, shipped and the controller tick; clock probes of the default clock build.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/abfold
mkdir -p $O
D=$R/go2_onnx_controller_amd/lib/diag
timeout -k 10 900 python3 -u -m pytest $R/tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo "gpu tests failed"; grep -E "FAILED|Error" $O/tests.log | head -20; tail -30 $O/tests.log; exit 1; }
tail -n 1 $O/tests.log
timeout -k 10 600 python3 $R/tools/ab.py --rounds 3 --out $O fold avt=avt 2>&1 | tee $O/ab_mlp512.txt || exit 1
timeout -k 10 600 python3 $R/tools/ab.py --rounds 2 --workload go2_gru_256_b4096 --out $O fold avt=avt 2>&1 | tee $O/ab_gru.txt || exit 1
timeout -k 10 600 python3 $R/tools/ab.py --rounds 2 --workload go2_lstm_256_b4096 --out $O fold avt=avt 2>&1 | tee $O/ab_lstm.txt || exit 1
timeout -k 10 600 python3 $R/tools/ab.py --rounds 2 --workload shipped_b4096 --out $O fold avt=avt 2>&1 | tee $O/ab_shipped.txt || exit 1
timeout -k 10 600 python3 $R/tools/ab.py --rounds 2 --ctl --workload shipped_b4096 --out $O fold avt=avt 2>&1 | tee $O/ab_ctl.txt || exit 1
export GO2PI_LIB=$D/libgo2pi_clock.so GO2PI_DIAG_STAMPS=1
timeout -k 10 120 python3 $R/tools/clock_probe.py --waves 4 > $O/clock_mlp512.json || exit 1
timeout -k 10 120 python3 $R/tools/clock_probe.py --waves 4 --ctl --model tests/golden/model.onnx > $O/clock_ctl.json || exit 1
for c in mlp512 ctl; do
  python3 -c "import json; d=json.load(open('$O/clock_$c.json')); print('$c', {k: d[k] for k in ('wg_cycles_median','wg_us_median','event_us_per_launch','wg_start_spread_us','wg_end_spread_us','phase_cycles_median','pipeline_layer1_subphases','ctl_assembly_blocks')})"
done
