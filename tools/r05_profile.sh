#!/bin/bash
# Round-5 profile pass (GPU box, repo root): rocprofv3 kernel stats + FETCH/WRITE PMC
# passes for mlp512 (configs[2]), GRU-256 one tick per launch and seq100 (configs[4]),
# the controller tick; the clock probes (GO2PI_DIAG_CLOCK build) of mlp512, the GRU-256
# tick and the controller tick; then the default bench line. Summarise with
# tools/summarize_prof.py --round r05.
set -o pipefail
mkdir -p gpurun_out
TAG=mlp512 STEPS=300 ARGS="--no-cpu --no-latency --no-ctl --no-gru" bash tools/profile.sh || exit 1
TAG=gru256 STEPS=100 ARGS="--no-cpu --no-latency --no-ctl --no-gru --workload go2_gru_256_b4096" bash tools/profile.sh || exit 1
TAG=gru256seq STEPS=40 ARGS="--no-cpu --no-latency --no-ctl --no-gru --workload go2_gru_256_b4096_seq100" bash tools/profile.sh || exit 1
TAG=ctl STEPS=50 ARGS="--no-cpu --no-gru" bash tools/profile.sh || exit 1
# keep what tools/summarize_prof.py reads (the per-dispatch traces would push gpurun_out
# past what the box copies back)
find gpurun_out -path '*prof_*' -type f ! -name 'run_kernel_stats.csv' ! -name 'run_counter_collection.csv' ! -name '*.log' -delete
echo profiles done
if [ -f go2_onnx_controller_amd/lib/diag/libgo2pi_clock.so ]; then
  export GO2PI_LIB=$PWD/go2_onnx_controller_amd/lib/diag/libgo2pi_clock.so GO2PI_DIAG_STAMPS=1
  timeout -k 10 120 python tools/clock_probe.py --waves 4 > gpurun_out/clock_mlp512.json || exit 1
  timeout -k 10 120 python tools/clock_probe.py --waves 4 --model go2_gru_256 > gpurun_out/clock_gru256.json || exit 1
  timeout -k 10 120 python tools/clock_probe.py --waves 4 --ctl --model tests/golden/model.onnx > gpurun_out/clock_ctl.json || exit 1
  unset GO2PI_LIB GO2PI_DIAG_STAMPS
  echo clocks done
fi
timeout -k 10 400 python bench.py > gpurun_out/bench_full.json 2> gpurun_out/bench_full.err || exit 1
cat gpurun_out/bench_full.json
# LSTM-256 lines (one tick per launch, 100 ticks per launch)
timeout -k 10 200 python bench.py --workload go2_lstm_256_b4096 --no-cpu --no-latency --no-ctl --no-gru > gpurun_out/bench_lstm256.json 2> gpurun_out/bench_lstm256.err || exit 1
timeout -k 10 200 python bench.py --workload go2_lstm_256_b4096_seq100 --no-cpu --no-latency --no-ctl --no-gru > gpurun_out/bench_lstm256_seq100.json 2> gpurun_out/bench_lstm256_seq100.err || exit 1
echo lstm done
