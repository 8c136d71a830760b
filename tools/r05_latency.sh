#!/bin/bash
# r05 batch-1 latency A/B on the GPU box: the drop-in ONNXActor::act() timed from C++
# (as the reference's main.cpp:38-42 times it) for the shipped model, alternating the
# r05 one-workgroup kernel (policy_act1_kernel: polling wave + 4 or 8 compute waves,
# GO2PI_A1_CW; one or two poll sweeps in flight, GO2PI_A1_DEPTH), the r04 1024-thread form
# (GO2PI_RES_R1W=1), the request ring in pinned host memory instead of BAR-mapped VRAM
# (GO2PI_REQ_HOST=1) and a launch per call (GO2PI_RESIDENT_MS=0);
# then, with a resclk build present, the request timeline (tools/res_timeline.py).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/lat
mkdir -p $O $R/build
L=$R/go2_onnx_controller_amd/lib
g++ -std=c++20 -O2 -I$R/include $R/tests/cpp/controller_shape.cpp -L$L -lonnx_actor -Wl,-rpath,$L -o $R/build/controller_shape || exit 1
M=$R/tests/golden/model.onnx
for round in 1 2 3; do
  [ -n "$SKIP_ACT" ] && break
  for v in ${VARIANTS:-c8d2 c8d1 c8d2host c4d2 r1w launch}; do
    case $v in
      c8d2host) env="GO2PI_A1_CW=8 GO2PI_REQ_HOST=1" ;;
      c4d2) env="GO2PI_A1_CW=4" ;;
      c4d1) env="GO2PI_A1_CW=4 GO2PI_A1_DEPTH=1" ;;
      c8d2) env="GO2PI_A1_CW=8" ;;
      c8d1) env="GO2PI_A1_CW=8 GO2PI_A1_DEPTH=1" ;;
      r1w) env="GO2PI_RES_R1W=1" ;;
      launch) env="GO2PI_RESIDENT_MS=0" ;;
    esac
    r=$(env $env timeout -k 10 60 $R/build/controller_shape $M lat 10000 1000 98 12) || { echo "lat $v failed: $r"; exit 1; }
    echo "round $round $v $(echo $r | tr '\n' ' ')" | tee -a $O/ab.txt
  done
done
# the batch-1 controller tick through the C ABI (tests/cpp/ctl_lat.c)
gcc -O2 -I$R/include $R/tests/cpp/ctl_lat.c -L$L -lgo2pi -Wl,-rpath,$L -o $R/build/ctl_lat || exit 1
for round in 1 2; do
  for v in ${CTL_VARIANTS:-a1 a1host r1w launch}; do
    case $v in
      a1) env=""; rm=100; x="" ;;
      a1min) env=""; rm=100; x=min ;;  # (only obs and action asked for)
      a1host) env="GO2PI_REQ_HOST=1"; rm=100; x="" ;;
      r1w) env="GO2PI_RES_R1W=1"; rm=100; x="" ;;
      r1wmin) env="GO2PI_RES_R1W=1"; rm=100; x=min ;;
      launch) env=""; rm=0; x="" ;;
    esac
    r=$(env $env timeout -k 10 60 $R/build/ctl_lat $M 10000 1000 $rm $x) || { echo "ctl_lat $v failed: $r"; exit 1; }
    echo "ctl round $round $v $(echo $r | tr '\n' ' ')" | tee -a $O/ab.txt
  done
done
if [ -f $L/diag/libgo2pi_resclk.so ]; then
  GO2PI_LIB=$L/diag/libgo2pi_resclk.so timeout -k 10 120 python3 $R/tools/res_timeline.py --model shipped --form one --ctl \
    --out $O/res_timeline_ctl.json > $O/res_timeline_ctl.log 2>&1 || { echo "ctl timeline failed"; tail -20 $O/res_timeline_ctl.log; exit 1; }
fi
if [ -f $L/diag/libgo2pi_resclk.so ]; then
  GO2PI_LIB=$L/diag/libgo2pi_resclk.so timeout -k 10 120 python3 $R/tools/res_timeline.py --model shipped --form one \
    --out $O/res_timeline_one.json > $O/res_timeline.log 2>&1 || { echo "timeline failed"; tail -20 $O/res_timeline.log; exit 1; }
  tail -30 $O/res_timeline_one.json
fi
echo "r05_latency ok"
