#!/bin/bash
# r05: the 8-wave lean kernel's parity (test_mlp512) under each issue-priority mode,
# then the lean controller tick A/B (tools/r05_ctl_ab.sh).
set -o pipefail
mkdir -p gpurun_out/w8
for pm in 0 1 2 3; do
  GO2PI_W8=1 GO2PI_W8_PRIO=$pm timeout -k 10 120 python3 -u -m pytest tests/test_gpu_parity.py -q --timeout 60 --timeout-method thread -k "mlp512" > gpurun_out/w8/pm$pm.log 2>&1
  echo "pm $pm rc=$? $(tail -1 gpurun_out/w8/pm$pm.log)"
done
bash tools/r05_ctl_ab.sh
