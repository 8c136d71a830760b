#!/bin/bash
# r05 A/B of the lean kernel at 4 waves against 8 waves (two per SIMD) and the 8-wave
# issue-priority modes (fused_impl.hpp w4_prio); the 8-wave parity tests first.
set -o pipefail
mkdir -p gpurun_out/w8
GO2PI_W8=1 GO2PI_W8_PRIO=${PM:-1} timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_pipeline.py -x -q --timeout 120 --timeout-method thread > gpurun_out/w8/tests.log 2>&1 || { echo "w8 tests failed"; tail -30 gpurun_out/w8/tests.log; exit 1; }
tail -2 gpurun_out/w8/tests.log
timeout -k 10 600 python3 tools/ab.py --rounds 3 ${VARIANTS:-w4 w8,GO2PI_W8=1 w8p1,GO2PI_W8=1,GO2PI_W8_PRIO=1 w8p2,GO2PI_W8=1,GO2PI_W8_PRIO=2 w8p3,GO2PI_W8=1,GO2PI_W8_PRIO=3} > gpurun_out/w8/ab.txt 2>&1 || { echo "ab failed"; tail -20 gpurun_out/w8/ab.txt; exit 1; }
cat gpurun_out/w8/ab.txt
