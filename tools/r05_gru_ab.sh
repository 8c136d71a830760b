#!/bin/bash
# r05: GRU / LSTM parity and the GRU-256 bench legs on the current build.
set -o pipefail
mkdir -p gpurun_out/gru
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_gru.py tests/test_gpu_lstm.py tests/test_gpu_resident.py -x -q --timeout 120 --timeout-method thread > gpurun_out/gru/tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/gru/tests.log; exit 1; }
tail -1 gpurun_out/gru/tests.log
for r in 1 2 3; do
  timeout -k 10 200 python3 -c "import bench, json; o = bench.gru_leg(0); print(json.dumps({k: (o[k]['us_per_tick'], o[k]['frac_fp32_peak']) for k in ('per_tick', 'seq100')}))" > gpurun_out/gru/leg$r.json 2> gpurun_out/gru/leg$r.err || { echo "gru leg failed"; tail -5 gpurun_out/gru/leg$r.err; exit 1; }
  echo "round $r $(cat gpurun_out/gru/leg$r.json)"
done
