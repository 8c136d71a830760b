#!/bin/bash
# Round 3: LSTM stage skips the all-zero x chunk of a 48-wide observation (ring from
# slot 1) vs the previous build (prev): LSTM + GRU parity, A/B.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/ab10
mkdir -p $O
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_lstm.py tests/test_gpu_gru.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 600 python3 tools/ab.py --rounds 2 --workload go2_lstm_256_b4096 --out $O new prev=prev || exit 1
timeout -k 10 600 python3 tools/ab.py --rounds 2 --steps 60 --workload go2_lstm_256_b4096_seq100 --out $O new prev=prev || exit 1
