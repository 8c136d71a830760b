#!/bin/bash
# Same-box A/B: shipped build vs the GO2PI_DIAG_PREFETCH variant, alternated twice.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/abp
mkdir -p $O
for rep in 1 2; do
  for v in default prefetch; do
    if [ $v = default ]; then unset GO2PI_LIB; else export GO2PI_LIB=$R/go2_onnx_controller_amd/lib/diag/libgo2pi_$v.so; fi
    for wl in go2_mlp_512_b4096 go2_gru_256_b4096; do
      timeout -k 10 120 python3 $R/bench.py --workload $wl --no-cpu --no-latency > $O/b_${v}_${wl}_$rep.json 2> $O/err || { echo "bench $v $wl failed"; tail $O/err; exit 1; }
      python3 -c "import json;d=json.load(open('$O/b_${v}_${wl}_$rep.json'));print('$rep $v $wl', d['kernel_us'], d.get('controller_tick',{}).get('tick_us'))"
    done
  done
done
