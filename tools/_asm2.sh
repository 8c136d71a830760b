#!/bin/bash
# one-off: the controller assembly run twice (GO2PI_DIAG_ASM2): cold vs warm pass cycles
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out/q
export GO2PI_LIB=$R/go2_onnx_controller_amd/lib/diag/libgo2pi_asm2_clock.so GO2PI_DIAG_STAMPS=1
timeout -k 10 120 python3 $R/tools/clock_probe.py --waves 4 --ctl --model tests/golden/model.onnx > $R/gpurun_out/q/clock_ctl_asm2.json && cat $R/gpurun_out/q/clock_ctl_asm2.json
