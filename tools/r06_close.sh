#!/bin/bash
# Round-6 closing measurements (GPU box, repo root): clock probes (GO2PI_DIAG_CLOCK build,
# start stamps at kernel entry) of mlp512, the GRU-256 tick and the controller tick; the
# launch probes (spin kernel, real kernel from C++); the default bench line and the
# recurrent lines; the batch-1 act() A/B and the wide kernel's request timeline.
set -o pipefail
O=gpurun_out/r06
mkdir -p $O
export GO2PI_LIB=$PWD/go2_onnx_controller_amd/lib/diag/libgo2pi_clock.so GO2PI_DIAG_STAMPS=1
timeout -k 10 120 python3 tools/clock_probe.py --waves 4 > $O/clock_mlp512.json || exit 1
timeout -k 10 120 python3 tools/clock_probe.py --waves 4 --model go2_gru_256 > $O/clock_gru256.json || exit 1
timeout -k 10 120 python3 tools/clock_probe.py --waves 4 --ctl --model tests/golden/model.onnx > $O/clock_ctl.json || exit 1
unset GO2PI_LIB GO2PI_DIAG_STAMPS
echo clocks done
[ -x tools/launch_probe.bin ] && { timeout -k 10 120 tools/launch_probe.bin > $O/launch_probe.txt 2>&1 || exit 1; }
M512=$(python3 -c "from go2_onnx_controller_amd import synth; print(synth.ensure_model('go2_mlp_512'))")
[ -x tools/batched_probe.bin ] && { timeout -k 10 120 tools/batched_probe.bin $M512 4096 1000 > $O/batched_probe.txt 2>&1 || exit 1; }
timeout -k 10 500 python3 bench.py > $O/bench_full.json 2> $O/bench_full.err || { tail -20 $O/bench_full.err; exit 1; }
cat $O/bench_full.json
for w in go2_gru_256_b4096 go2_lstm_256_b4096 go2_lstm_256_b4096_seq100; do
  timeout -k 10 300 python3 bench.py --workload $w --no-cpu --no-latency --no-ctl --no-gru > $O/bench_$w.json 2> $O/bench_$w.err || { tail -20 $O/bench_$w.err; exit 1; }
done
echo benches done
SEL_SKIP=1 bash tools/r06_wide.sh || exit 1
