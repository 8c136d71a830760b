# Resident batch-1 path: GPU tests, then host->host latency per mode (same box).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_resident.py -x -v --timeout 120 --timeout-method thread > gpurun_out/resident_tests.log 2>&1 || { tail -40 gpurun_out/resident_tests.log; exit 1; }
tail -3 gpurun_out/resident_tests.log
for m in go2_mlp_512 shipped; do
  timeout -k 10 120 python3 tools/latency_probe.py --model $m --iters 5000 || exit 1
  timeout -k 10 120 python3 tools/latency_probe.py --model $m --iters 5000 --resident-ms 200 || exit 1
  GO2PI_RES_TILED0=1 timeout -k 10 120 python3 tools/latency_probe.py --model $m --iters 5000 --resident-ms 200 || exit 1
done
timeout -k 10 120 python3 tools/latency_probe.py --model go2_mlp_512 --iters 5000 --resident-ms 200 --batch 8 || exit 1
timeout -k 10 120 python3 tools/latency_probe.py --model go2_mlp_512 --iters 5000 --batch 8 || exit 1
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_controller.py -x -q --timeout 120 --timeout-method thread > gpurun_out/ctl_tests.log 2>&1 || { tail -40 gpurun_out/ctl_tests.log; exit 1; }
tail -2 gpurun_out/ctl_tests.log
timeout -k 10 300 python3 bench.py --no-cpu > gpurun_out/bench_rc.json 2> gpurun_out/bench_rc.err || { tail -20 gpurun_out/bench_rc.err; exit 1; }
cat gpurun_out/bench_rc.json
