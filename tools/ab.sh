#!/bin/bash
# A/B of the batched kernel's schedule variants on the GPU box (repo root):
# smoke parity, bench per library variant, clock probe per variant, then the GPU tests.
# Variants (Makefile diag target, -DGO2PI_DIAG_<NAME>): default (k-outer MFMA
# order + a workgroup barrier per layer), handoff (per-wave LDS flag hand-off
# between wide layers), tileouter (the previous MFMA order); *_clock adds stamps.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/ab
mkdir -p $O
D=$R/go2_onnx_controller_amd/lib/diag
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
echo "smoke ok"
for v in default handoff; do
  if [ $v = default ]; then unset GO2PI_LIB; else export GO2PI_LIB=$D/libgo2pi_$v.so; fi
  for wl in go2_mlp_512_b4096 go2_gru_256_b4096 shipped_b4096; do
    timeout -k 10 120 python3 $R/bench.py --workload $wl --no-cpu --no-latency --no-ctl > $O/b_${v}_$wl.json 2> $O/b_${v}_$wl.err || { echo "bench $v $wl failed"; exit 1; }
    python3 -c "import json;d=json.load(open('$O/b_${v}_$wl.json'));print('$v $wl', d['kernel_us'], d['roofline']['frac'])"
  done
done
unset GO2PI_LIB
export GO2PI_DIAG_STAMPS=1
for v in clock handoff_clock tileouter_clock; do
  GO2PI_LIB=$D/libgo2pi_$v.so timeout -k 10 120 python3 $R/tools/clock_probe.py > $O/clock_$v.json 2> $O/clock_$v.err || { echo "clock $v failed"; exit 1; }
  python3 -c "import json;d=json.load(open('$O/clock_$v.json'));print('$v', d['wg_cycles_median'], d['event_us_per_launch'], d['phase_cycles_median'])"
done
unset GO2PI_DIAG_STAMPS
timeout -k 10 900 python3 -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -5 $O/tests.log
exit $rc
