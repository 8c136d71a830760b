#!/bin/bash
# r06 GPU pass (repo root on the box): the GPU test suite, the launch-overhead probe
# (tools/launch_probe.hip), clock probes of the batched mlp512 kernel and the
# controller tick (GO2PI_DIAG_CLOCK build), then the default bench line. Each step
# under its own time limit; a failing step ends the script.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/p
mkdir -p $O
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 1100 python3 -u -m pytest $R/tests -m gpu -x -q --timeout 120 --timeout-method thread ${SEL:-} > $O/tests.log 2>&1 || { echo "gpu tests failed"; grep -E "FAILED|Error" $O/tests.log | head -20; tail -40 $O/tests.log; exit 1; }
  tail -2 $O/tests.log
fi
if [ -x $R/tools/launch_probe.bin ]; then
  timeout -k 10 120 $R/tools/launch_probe.bin > $O/launch_probe.txt 2>&1 || { echo "launch_probe failed"; cat $O/launch_probe.txt; exit 1; }
  cat $O/launch_probe.txt
fi
if [ -f $R/go2_onnx_controller_amd/lib/diag/libgo2pi_clock.so ]; then
  export GO2PI_LIB=$R/go2_onnx_controller_amd/lib/diag/libgo2pi_clock.so GO2PI_DIAG_STAMPS=1
  timeout -k 10 120 python3 $R/tools/clock_probe.py --waves 4 > $O/clock_mlp512.json || exit 1
  timeout -k 10 120 python3 $R/tools/clock_probe.py --waves 4 --ctl --model tests/golden/model.onnx > $O/clock_ctl.json || exit 1
  unset GO2PI_LIB GO2PI_DIAG_STAMPS
  python3 -c "import json; d=json.load(open('$O/clock_mlp512.json')); print({k: d[k] for k in ('wg_us_median','launch_span_us','event_us_per_launch','wg_start_spread_us','wg_end_spread_us','phase_cycles_median')})"
fi
[ -n "$NO_BENCH" ] || { timeout -k 10 600 python3 $R/bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 1; }; cat $O/bench.json; }
if [ -z "$NO_BENCH" ]; then  # the recurrent one-tick lines (lean GRU / LSTM ticks)
  for w in go2_gru_256_b4096 go2_lstm_256_b4096; do
    timeout -k 10 300 python3 $R/bench.py --workload $w --no-cpu --no-latency --no-ctl --no-gru > $O/bench_$w.json 2> $O/bench_$w.err || { echo "bench $w failed"; tail -20 $O/bench_$w.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/bench_$w.json')); print('$w', d['ms_per_step'], d['roofline']['frac'], d['config'])"
  done
fi
echo "r06_pass ok"
