#!/bin/bash
# r06 A/B of the hidden-layer epilogue (tools/build_variant.sh builds): MFMA accumulators in
# VGPRs (-amdgpu-mfma-vgpr-form: no accvgpr reads in front of the Elu), the Elu select as an
# integer min (GO2PI_ELU_IMIN), both; parity of the variants first.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/abepi
mkdir -p $O
for v in ${VARS:-vgpr imin vimin}; do
  GO2PI_LIB=$R/go2_onnx_controller_amd/lib/diag/libgo2pi_$v.so timeout -k 10 300 python3 -u -m pytest $R/tests/test_gpu_parity.py $R/tests/test_gpu_gru.py $R/tests/test_gpu_boundary.py -x -q --timeout 120 --timeout-method thread > $O/tests_$v.log 2>&1 || { echo "tests $v failed"; tail -30 $O/tests_$v.log; exit 1; }
  echo "$v: $(tail -n 1 $O/tests_$v.log)"
done
timeout -k 10 600 python3 $R/tools/ab.py --rounds ${ROUNDS:-3} --out $O base $(for v in ${VARS:-vgpr imin vimin}; do echo -n "$v=$v "; done) 2>&1 | tee $O/ab_mlp512.txt || exit 1
[ -n "$NO_GRU" ] || timeout -k 10 600 python3 $R/tools/ab.py --rounds 2 --workload go2_gru_256_b4096 --out $O base $(for v in ${VARS:-vgpr imin vimin}; do echo -n "$v=$v "; done) 2>&1 | tee $O/ab_gru.txt || exit 1
for c in ${CLK:-clock}; do  # per-XCD spreads and phases of the batched kernel (clock builds)
  GO2PI_LIB=$R/go2_onnx_controller_amd/lib/diag/libgo2pi_$c.so GO2PI_DIAG_STAMPS=1 timeout -k 10 120 python3 $R/tools/clock_probe.py --waves 4 > $O/clock_$c.json || exit 1
  python3 -c "import json; d=json.load(open('$O/clock_$c.json')); print('$c', {k: d[k] for k in ('wg_cycles_median','wg_us_median','event_us_per_launch','wg_start_spread_us','wg_end_spread_us','phase_cycles_median','pipeline_layer1_subphases','ctl_assembly_blocks')})"
done
