#!/bin/bash
# r06: the lean controller tick's whole-row assembly (ctl_assemble_rows): controller tests,
# tick A/B against avt (the r06 build before it), the tick's clock probe.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/abctl
mkdir -p $O
D=$R/go2_onnx_controller_amd/lib/diag
timeout -k 10 400 python3 -u -m pytest $R/tests/test_gpu_controller.py $R/tests/test_gpu_boundary.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error" $O/tests.log | head -20; tail -30 $O/tests.log; exit 1; }
tail -n 1 $O/tests.log
timeout -k 10 600 python3 $R/tools/ab.py --rounds 3 --ctl --workload shipped_b4096 --out $O new base7=base7 2>&1 | tee $O/ab_ctl.txt || exit 1
export GO2PI_LIB=$D/libgo2pi_clock.so GO2PI_DIAG_STAMPS=1
timeout -k 10 120 python3 $R/tools/clock_probe.py --waves 4 --ctl --model tests/golden/model.onnx > $O/clock_ctl.json || exit 1
python3 -c "import json; d=json.load(open('$O/clock_ctl.json')); print({k: d[k] for k in ('wg_cycles_median','wg_us_median','launch_span_us','event_us_per_launch','phase_cycles_median','ctl_assembly_blocks')})"


