#!/bin/bash
# r05: the 8-wave lean kernel's parity (test_mlp512) under priority / offset modes, then
# the A/B of 4 waves against 8 waves with those modes (tools/ab.py).
set -o pipefail
mkdir -p gpurun_out/w8
for pm in 6 9; do
  GO2PI_W8=1 GO2PI_W8_PRIO=$pm timeout -k 10 120 python3 -u -m pytest tests/test_gpu_parity.py -q --timeout 60 --timeout-method thread -k "mlp512" > gpurun_out/w8/pm$pm.log 2>&1
  echo "pm $pm rc=$? $(tail -1 gpurun_out/w8/pm$pm.log)"
done
timeout -k 10 900 python3 tools/ab.py --rounds 3 ${VARIANTS:-w4 w8p2,GO2PI_W8=1,GO2PI_W8_PRIO=2 w8d1,GO2PI_W8=1,GO2PI_W8_PRIO=4 w8d2,GO2PI_W8=1,GO2PI_W8_PRIO=8 w8p2d1,GO2PI_W8=1,GO2PI_W8_PRIO=6 w8p2d2,GO2PI_W8=1,GO2PI_W8_PRIO=10 w8p1d1,GO2PI_W8=1,GO2PI_W8_PRIO=5} > gpurun_out/w8/ab.txt 2>&1 || { echo "ab failed"; tail -20 gpurun_out/w8/ab.txt; exit 1; }
tail -8 gpurun_out/w8/ab.txt
