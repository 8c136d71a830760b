# Clock-probe ablations of the lean batched kernel (mlp512): stock, no weight loads,
# no MFMAs, ring depth 2, epilogue woven into the own phase. Diagnostics only.
set -o pipefail
mkdir -p gpurun_out/diag3
export GO2PI_DIAG_STAMPS=1
for v in clock noload_clock nomfma_clock rd2_clock weave_clock; do
  GO2PI_LIB=$PWD/go2_onnx_controller_amd/lib/diag/libgo2pi_$v.so timeout -k 10 120 python tools/clock_probe.py --waves 4 > gpurun_out/diag3/$v.json 2> gpurun_out/diag3/$v.err || { echo "$v failed"; exit 1; }
  python3 -c "
import json,sys; d=json.load(open('gpurun_out/diag3/$v.json')); print('$v', d['wg_cycles_median'], round(d['event_us_per_launch'],2), d['clock_ghz_median'], d['phase_cycles_median'], d['pipeline_layer1_subphases'].get('0'))"
done
