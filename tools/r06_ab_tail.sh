#!/bin/bash
# r06 A/B: the lean kernels' tail (one store sequence, no per-activation copies) on top of
# the VGPR-form MFMA + integer-min Elu epilogue, for mlp512, the shipped model and the
# controller tick; parity of the variants first; clock probes of the avtclk build.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/abtail
mkdir -p $O
D=$R/go2_onnx_controller_amd/lib/diag
for v in ${VARS:-vt avt}; do
  GO2PI_LIB=$D/libgo2pi_$v.so timeout -k 10 400 python3 -u -m pytest $R/tests/test_gpu_parity.py $R/tests/test_gpu_gru.py $R/tests/test_gpu_boundary.py $R/tests/test_gpu_controller.py $R/tests/test_gpu_lstm.py -x -q --timeout 120 --timeout-method thread > $O/tests_$v.log 2>&1 || { echo "tests $v failed"; tail -30 $O/tests_$v.log; exit 1; }
  echo "$v: $(tail -n 1 $O/tests_$v.log)"
done
timeout -k 10 600 python3 $R/tools/ab.py --rounds 3 --out $O base vnc=vnc vt=vt avt=avt 2>&1 | tee $O/ab_mlp512.txt || exit 1
timeout -k 10 600 python3 $R/tools/ab.py --rounds 3 --workload shipped_b4096 --out $O base avt=avt 2>&1 | tee $O/ab_shipped.txt || exit 1
timeout -k 10 600 python3 $R/tools/ab.py --rounds 3 --ctl --workload shipped_b4096 --out $O base avt=avt 2>&1 | tee $O/ab_ctl.txt || exit 1
timeout -k 10 600 python3 $R/tools/ab.py --rounds 2 --workload go2_gru_256_b4096 --out $O base avt=avt 2>&1 | tee $O/ab_gru.txt || exit 1
timeout -k 10 600 python3 $R/tools/ab.py --rounds 2 --workload go2_lstm_256_b4096 --out $O base avt=avt 2>&1 | tee $O/ab_lstm.txt || exit 1
export GO2PI_LIB=$D/libgo2pi_avtclk.so GO2PI_DIAG_STAMPS=1
timeout -k 10 120 python3 $R/tools/clock_probe.py --waves 4 > $O/clock_mlp512.json || exit 1
timeout -k 10 120 python3 $R/tools/clock_probe.py --waves 4 --ctl --model tests/golden/model.onnx > $O/clock_ctl.json || exit 1
for c in mlp512 ctl; do
  python3 -c "import json; d=json.load(open('$O/clock_$c.json')); print('$c', {k: d[k] for k in ('wg_cycles_median','wg_us_median','event_us_per_launch','wg_start_spread_us','wg_end_spread_us','phase_cycles_median','pipeline_layer1_subphases','ctl_assembly_blocks')})"
done
