#!/bin/bash
# r05: GRU / LSTM / pipeline / resident parity, then the GRU-256 bench legs, the lean GRU
# tick (policy_gru_kernel) alternated with the general body (GO2PI_GRU_GENERAL=1).
set -o pipefail
mkdir -p gpurun_out/gru
GO2PI_GRU_LEAN=1 timeout -k 10 400 python3 -u -m pytest tests/test_gpu_gru.py tests/test_gpu_replay.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/gru/tests_lean.log 2>&1 || { echo "lean tests failed"; tail -30 gpurun_out/gru/tests_lean.log; exit 1; }
tail -1 gpurun_out/gru/tests_lean.log
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_gru.py tests/test_gpu_lstm.py tests/test_gpu_pipeline.py tests/test_gpu_resident.py -x -q --timeout 120 --timeout-method thread > gpurun_out/gru/tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/gru/tests.log; exit 1; }
tail -1 gpurun_out/gru/tests.log
for r in 1 2 3; do
  for v in lean general; do
    if [ $v = general ]; then unset GO2PI_GRU_LEAN; else export GO2PI_GRU_LEAN=1; fi
    timeout -k 10 200 python3 -c "import bench, json; o = bench.gru_leg(0); print(json.dumps({k: (o[k]['us_per_tick'], o[k]['frac_fp32_peak']) for k in ('per_tick', 'seq100')}), o['kernel'])" > gpurun_out/gru/$v$r.json 2> gpurun_out/gru/$v$r.err || { echo "gru leg failed"; tail -5 gpurun_out/gru/$v$r.err; exit 1; }
    echo "round $r $v $(cat gpurun_out/gru/$v$r.json)"
  done
done
