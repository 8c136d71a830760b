#!/bin/bash
# r06: what a batched launch pays outside its workgroups, measured three ways on one box:
# the spin-kernel probe (tools/launch_probe.bin), the real kernel timed from C++ on a plain
# HIP stream (tools/batched_probe.bin), and the clock probes with start stamps taken at
# kernel entry (GO2PI_ENTRY_CLOCK) for mlp512, the controller tick and the GRU-256 tick.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/launch
mkdir -p $O
M512=$(python3 -c "import sys; sys.path.insert(0, '$R'); from go2_onnx_controller_amd import synth; print(synth.ensure_model('go2_mlp_512'))")
MGRU=$(python3 -c "import sys; sys.path.insert(0, '$R'); from go2_onnx_controller_amd import synth; print(synth.ensure_model('go2_gru_256'))")
timeout -k 10 120 $R/tools/launch_probe.bin > $O/launch_probe.txt 2>&1 || { cat $O/launch_probe.txt; exit 1; }
head -n 3 $O/launch_probe.txt
for m in $M512 $MGRU $R/tests/golden/model.onnx; do
  timeout -k 10 120 $R/tools/batched_probe.bin $m 4096 1000 2>&1 | tee -a $O/batched_probe.txt || exit 1
done
export GO2PI_LIB=$R/go2_onnx_controller_amd/lib/diag/libgo2pi_clock.so GO2PI_DIAG_STAMPS=1
timeout -k 10 120 python3 $R/tools/clock_probe.py --waves 4 > $O/clock_mlp512.json || exit 1
timeout -k 10 120 python3 $R/tools/clock_probe.py --waves 4 --ctl --model tests/golden/model.onnx > $O/clock_ctl.json || exit 1
timeout -k 10 120 python3 $R/tools/clock_probe.py --waves 4 --model go2_gru_256 > $O/clock_gru256.json || exit 1
for c in mlp512 ctl gru256; do
  python3 -c "import json; d=json.load(open('$O/clock_$c.json')); print('$c', {k: d[k] for k in ('wg_cycles_median','wg_us_median','launch_span_us','event_us_per_launch','wg_start_spread_us','wg_end_spread_us','phase_cycles_median','init_subphases')}, 'event-span', round(d['event_us_per_launch'] - d['launch_span_us'], 3))"
done
