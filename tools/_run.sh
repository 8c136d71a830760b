# Round profile pass (GPU box, repo root): rocprofv3 stats + PMC for mlp512, gru256 and
# the controller tick, the full bench line, and clock probes. Summarise afterwards with
# tools/summarize_prof.py --round rNN.
set -o pipefail
mkdir -p gpurun_out
TAG=mlp512 STEPS=300 bash tools/profile.sh || exit 1
TAG=gru256 STEPS=200 ARGS="--no-cpu --no-latency --no-ctl --workload go2_gru_256_b4096" bash tools/profile.sh || exit 1
TAG=ctl STEPS=50 ARGS="--no-cpu" bash tools/profile.sh || exit 1
timeout -k 10 300 python bench.py > gpurun_out/bench_full.json 2> gpurun_out/bench_full.err || exit 1
export GO2PI_LIB=$PWD/go2_onnx_controller_amd/lib/diag/libgo2pi_clock.so GO2PI_DIAG_STAMPS=1
timeout -k 10 120 python tools/clock_probe.py --waves 4 > gpurun_out/clock_mlp512.json || exit 1
timeout -k 10 120 python tools/clock_probe.py --waves 4 --model go2_gru_256 > gpurun_out/clock_gru256.json || exit 1
timeout -k 10 120 python tools/clock_probe.py --waves 4 --model tests/golden/model.onnx > gpurun_out/clock_shipped.json || exit 1
timeout -k 10 120 python tools/clock_probe.py --waves 4 --model tests/golden/model.onnx --ctl > gpurun_out/clock_ctl.json || exit 1
echo done
