# Round-3 profile pass (GPU box, repo root): rocprofv3 kernel stats + FETCH/WRITE PMC
# passes for mlp512 (configs[2]), GRU-256 seq100 (configs[4]) and the controller tick,
# then the default bench line. Summarise with tools/summarize_prof.py --round r03.
set -o pipefail
mkdir -p gpurun_out
TAG=mlp512 STEPS=300 ARGS="--no-cpu --no-latency --no-ctl --no-gru" bash tools/profile.sh || exit 1
TAG=gru256seq STEPS=40 ARGS="--no-cpu --no-latency --no-ctl --no-gru --workload go2_gru_256_b4096_seq100" bash tools/profile.sh || exit 1
TAG=ctl STEPS=50 ARGS="--no-cpu --no-gru" bash tools/profile.sh || exit 1
timeout -k 10 400 python bench.py > gpurun_out/bench_full.json 2> gpurun_out/bench_full.err || exit 1
echo bench done
export GO2PI_LIB=$PWD/go2_onnx_controller_amd/lib/diag/libgo2pi_clock.so GO2PI_DIAG_STAMPS=1
timeout -k 10 120 python tools/clock_probe.py --waves 4 > gpurun_out/clock_mlp512.json || exit 1
timeout -k 10 120 python tools/clock_probe.py --waves 4 --model go2_gru_256 > gpurun_out/clock_gru256.json || exit 1
echo clocks done
