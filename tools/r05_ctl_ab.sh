#!/bin/bash
# r05 A/B of the 4096-robot controller tick: the lean tick kernel (policy_mlp_ctl_kernel)
# against the general body (GO2PI_CTL_GENERAL=1), alternated; the controller tests first.
set -o pipefail
mkdir -p gpurun_out/ctl
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_controller.py -x -q --timeout 120 --timeout-method thread > gpurun_out/ctl/tests.log 2>&1 || { echo "ctl tests failed"; tail -30 gpurun_out/ctl/tests.log; exit 1; }
tail -2 gpurun_out/ctl/tests.log
for r in 1 2 3; do
  for v in lean general; do
    if [ $v = general ]; then export GO2PI_CTL_GENERAL=1; else unset GO2PI_CTL_GENERAL; fi
    timeout -k 10 120 python3 -c "import bench, json; o = bench.controller_leg(0, iters=2000); print(json.dumps({k: o[k] for k in ('tick_us', 'policy_only_us', 'b1_tick_p50_us')}))" > gpurun_out/ctl/$v.$r.json 2> gpurun_out/ctl/$v.$r.err || { echo "ctl leg $v failed"; tail -20 gpurun_out/ctl/$v.$r.err; exit 1; }
    echo "round $r $v $(cat gpurun_out/ctl/$v.$r.json)"
  done
done
