# Development GPU pass: every GPU test, batch-1 latency per mode, the default bench line.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/ -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/tests.log 2>&1 || { tail -40 gpurun_out/tests.log; exit 1; }
tail -2 gpurun_out/tests.log
for m in go2_mlp_512 shipped; do
  timeout -k 10 120 python3 tools/latency_probe.py --model $m --iters 5000 || exit 1
  timeout -k 10 120 python3 tools/latency_probe.py --model $m --iters 5000 --resident-ms 200 || exit 1
done
for b in 4 8; do
  timeout -k 10 120 python3 tools/latency_probe.py --model go2_mlp_512 --iters 3000 --batch $b || exit 1
  timeout -k 10 120 python3 tools/latency_probe.py --model go2_mlp_512 --iters 3000 --batch $b --resident-ms 200 || exit 1
done
timeout -k 10 300 python3 bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
