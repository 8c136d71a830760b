set -o pipefail
R=$(pwd)
WAVES="8 16" bash tools/gpu_check.sh || { grep -E "FAIL|Error|error" gpurun_out/tests.log | head -20; exit 1; }
for v in clock noload_clock; do
for w in 8 16; do
  GO2PI_LIB=$R/go2_onnx_controller_amd/lib/diag/libgo2pi_$v.so timeout -k 10 120 python3 tools/clock_probe.py --waves $w --seconds 0.5 2>/dev/null | python3 -c "import json,sys;d=json.load(sys.stdin);print('$v w$w',d['wg_cycles_median'],d['phase_cycles_median'])" || exit 1
done
done
