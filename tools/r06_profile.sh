#!/bin/bash
# Round-6 profile pass (GPU box, repo root): the GPU test suite, then rocprofv3 kernel
# stats + FETCH/WRITE PMC passes for mlp512 (configs[2]), GRU-256 one tick per launch and
# seq100 (configs[4]), LSTM-256 one tick per launch and the controller tick. Summarise
# with tools/summarize_prof.py --round r06 (tools/r06_close.sh runs the clocks and bench).
set -o pipefail
mkdir -p gpurun_out/r06
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r06/tests.log 2>&1 || { echo "gpu tests failed"; grep -E "FAILED|Error|Timeout" gpurun_out/r06/tests.log | head -20; tail -20 gpurun_out/r06/tests.log; exit 1; }
tail -n 1 gpurun_out/r06/tests.log
TAG=mlp512 STEPS=300 ARGS="--no-cpu --no-latency --no-ctl --no-gru" bash tools/profile.sh || exit 1
TAG=gru256 STEPS=100 ARGS="--no-cpu --no-latency --no-ctl --no-gru --workload go2_gru_256_b4096" bash tools/profile.sh || exit 1
TAG=gru256seq STEPS=40 ARGS="--no-cpu --no-latency --no-ctl --no-gru --workload go2_gru_256_b4096_seq100" bash tools/profile.sh || exit 1
TAG=lstm256 STEPS=100 ARGS="--no-cpu --no-latency --no-ctl --no-gru --workload go2_lstm_256_b4096" bash tools/profile.sh || exit 1
TAG=ctl STEPS=50 ARGS="--no-cpu --no-gru" bash tools/profile.sh || exit 1
find gpurun_out -path '*prof_*' -type f ! -name 'run_kernel_stats.csv' ! -name 'run_counter_collection.csv' ! -name '*.log' -delete
echo profiles done
