#!/bin/bash
# r06: the lean recurrent tick without the hidden-row carry after its last tick, against
# base8: GRU / LSTM tests, A/B on the GRU-256 and LSTM-256 ticks.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/abgru
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest $R/tests/test_gpu_gru.py $R/tests/test_gpu_lstm.py $R/tests/test_gpu_resident.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|Timeout" $O/tests.log | head -20; tail -20 $O/tests.log; exit 1; }
tail -n 1 $O/tests.log
timeout -k 10 600 python3 $R/tools/ab.py --rounds 3 --workload go2_gru_256_b4096 --out $O nocarry base8=base8 2>&1 | tee $O/ab_gru.txt || exit 1
timeout -k 10 600 python3 $R/tools/ab.py --rounds 2 --workload go2_lstm_256_b4096 --out $O nocarry base8=base8 2>&1 | tee $O/ab_lstm.txt || exit 1
