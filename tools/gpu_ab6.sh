#!/bin/bash
# Round 3: epilogue with one AGPR read per element vs the previous build (prev): parity, A/B.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/ab6
D=$R/go2_onnx_controller_amd/lib/diag
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_pipeline.py tests/test_gpu_parity.py tests/test_gpu_boundary.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo "parity failed"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 600 python3 tools/ab.py --rounds 3 --out $O new prev=prev || exit 1
timeout -k 10 600 python3 tools/ab.py --rounds 2 --workload shipped_b4096 --out $O new prev=prev || exit 1
