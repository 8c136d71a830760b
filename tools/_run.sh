set -o pipefail
timeout -k 10 600 python -m pytest tests/ -m gpu -q -x > gpurun_out/tests.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/tests.log; [ $rc = 0 ] || { grep -E "^E |FAILED" gpurun_out/tests.log | head; exit 1; }
for a in "--model tiny" "" "--model shipped"; do
  timeout -k 10 120 python3 tools/latency_probe.py $a 2>/dev/null || exit 1
done
timeout -k 10 120 ./build/controller_shape tests/golden/model.onnx ticks 5000 | tail -1
