set -o pipefail
R=$(pwd)
timeout -k 10 600 python -m pytest tests/ -m gpu -q -x > gpurun_out/tests.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/tests.log; [ $rc = 0 ] || { grep -E "^E |FAILED" gpurun_out/tests.log | head; exit 1; }
GO2PI_LIB=$R/go2_onnx_controller_amd/lib/diag/libgo2pi_clock.so timeout -k 10 120 python3 tools/clock_probe.py --waves 8 --seconds 0.5 2>/dev/null | python3 -c "
import json,sys;d=json.load(sys.stdin);print(d['wg_cycles_median'],d['phase_cycles_median'])
m=d['layer1_wave_marks']; print('  wave0',[round(x) for x in m['0']], 'wave4', [round(x) for x in m['4']])" || exit 1
for i in 1 2 3; do timeout -k 10 300 python bench.py --no-cpu --no-latency 2>/dev/null | python3 -c "import json,sys;d=json.load(sys.stdin);print(d['value'],d['kernel_us'],d['roofline']['frac'])"; done
