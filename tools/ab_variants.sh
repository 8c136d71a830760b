#!/bin/bash
# Same-box A/B of batched-kernel variants (GPU box, repo root). Each round
# alternates the variants so box drift hits them all alike.
#   VARIANTS: library names ('default' = lib/libgo2pi.so, else lib/diag/libgo2pi_<v>.so)
#   WAVES:    waves per workgroup to try with every variant
#   CLOCKS:   *_clock variants for the in-kernel clock probe
#   PARITY:   variants whose GPU parity tests run (GO2PI_LIB pointed at them)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/ab
mkdir -p $O
D=$R/go2_onnx_controller_amd/lib/diag
WL=${WL:-go2_mlp_512_b4096}
libof() { if [ "$1" = default ]; then echo $R/go2_onnx_controller_amd/lib/libgo2pi.so; else echo $D/libgo2pi_$1.so; fi; }
[ "${VARIANTS:-}" = none ] && ROUNDS=skip
for rnd in ${ROUNDS:-1 2}; do
  [ "$rnd" = skip ] && break
  for v in ${VARIANTS:-default}; do
    for w in ${WAVES:-8}; do
      for wl in ${WLS:-$WL}; do
        f=$O/b_${v}_w${w}_${wl}_$rnd
        GO2PI_LIB=$(libof $v) timeout -k 10 180 python3 $R/bench.py --workload $wl --waves $w --no-cpu --no-latency --steps ${STEPS:-400} $([ -z "$CTLLEG" ] && echo --no-ctl) > $f.json 2> $f.err || { echo "bench $v w$w $wl failed"; tail -5 $f.err; exit 1; }
        python3 -c "import json;d=json.load(open('$f.json'));print('round $rnd $v waves $w $wl', d['kernel_us'], d['roofline']['frac'], d.get('controller_tick', ''))"
      done
    done
  done
done
export GO2PI_DIAG_STAMPS=1
for v in ${CLOCKS:-}; do
  for w in ${CLOCK_WAVES:-8}; do
    GO2PI_LIB=$D/libgo2pi_$v.so timeout -k 10 120 python3 $R/tools/clock_probe.py --model ${MODEL:-go2_mlp_512} --waves $w > $O/clock_${v}_w$w.json 2> $O/clock_${v}_w$w.err || { echo "clock $v failed"; tail -5 $O/clock_${v}_w$w.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/clock_${v}_w$w.json'));print('$v waves $w', d['wg_cycles_median'], d['event_us_per_launch'], d['phase_cycles_median']); print('   layer1 marks', d['layer1_wave_marks'], 'sub', d.get('pipeline_layer1_subphases'), 'init', d.get('init_subphases'), 'gru', d.get('gru_stage'))"
  done
done
unset GO2PI_DIAG_STAMPS
for v in ${PARITY:-}; do
  GO2PI_LIB=$(libof $v) timeout -k 10 600 python3 -u -m pytest tests/ -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests_$v.log 2>&1 || { echo "gpu tests failed with $v"; tail -30 $O/tests_$v.log; exit 1; }
  echo "parity $v: $(tail -1 $O/tests_$v.log)"
done
echo "ab ok"
