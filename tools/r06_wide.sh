#!/bin/bash
# r06 GPU pass for the wide-policy resident kernel (resident_wide.hip): its parity tests,
# then batch-1 ONNXActor::act() timed from C++ (as the reference's main.cpp:38-42 times
# it) for the 48->512^3->12 policy (BASELINE configs[1]) in three alternated rounds:
# the wide kernel (default), the r03 multi-workgroup kernel (GO2PI_RES_MULTI=1), the
# shipped model (act1) beside them; then the request timeline (resclk build).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/wide
mkdir -p $O $R/build
L=$R/go2_onnx_controller_amd/lib
[ -n "$SEL_SKIP" ] || timeout -k 10 600 python3 -u -m pytest $R/tests/test_gpu_resident.py -x -v --timeout 120 --timeout-method thread \
  -k "${SEL:-wide or ring or mlp512 or two_engines or destroy or interleaved or prologue}" > $O/tests.log 2>&1 \
  || { echo "tests failed"; grep -E "FAILED|Error|assert" $O/tests.log | head -30; tail -30 $O/tests.log; exit 1; }
[ -n "$SEL_SKIP" ] || tail -3 $O/tests.log
g++ -std=c++20 -O2 -I$R/include $R/tests/cpp/controller_shape.cpp -L$L -lonnx_actor -Wl,-rpath,$L -o $R/build/controller_shape || exit 1
M512=$(python3 -c "import sys; sys.path.insert(0, '$R'); from go2_onnx_controller_amd import synth; print(synth.ensure_model('go2_mlp_512'))")
for round in 1 2 3; do
  for v in wide multi shipped; do
    case $v in
      wide) env=""; m=$M512; i=48 ;;
      multi) env="GO2PI_RES_MULTI=1"; m=$M512; i=48 ;;
      shipped) env=""; m=$R/tests/golden/model.onnx; i=98 ;;
    esac
    r=$(env $env timeout -k 10 60 $R/build/controller_shape $m lat 10000 1000 $i 12) || { echo "lat $v failed: $r"; exit 1; }
    echo "round $round $v $(echo $r | tr '\n' ' ')" | tee -a $O/ab.txt
  done
done
if [ -f $L/diag/libgo2pi_resclk.so ]; then
  GO2PI_LIB=$L/diag/libgo2pi_resclk.so timeout -k 10 120 python3 $R/tools/res_timeline.py --model go2_mlp_512 --form wide \
    --out $O/res_timeline_wide.json > $O/res_timeline.log 2>&1 || { echo "timeline failed"; tail -20 $O/res_timeline.log; exit 1; }
  cat $O/res_timeline_wide.json
fi
echo "r06_wide ok"
