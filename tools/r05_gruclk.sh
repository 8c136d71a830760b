#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/probe
export GO2PI_LIB=$PWD/go2_onnx_controller_amd/lib/diag/libgo2pi_clock.so GO2PI_DIAG_STAMPS=1
timeout -k 10 120 python3 tools/clock_probe.py --waves 4 --model go2_gru_256 > gpurun_out/probe/clock_gru256.json && python3 -c "import json; d = json.load(open('gpurun_out/probe/clock_gru256.json')); print(d['gru_stage'], d['init_subphases'])"
