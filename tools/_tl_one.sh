set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out/lat
GO2PI_LIB=$R/go2_onnx_controller_amd/lib/diag/libgo2pi_resclk.so timeout -k 10 120 python3 $R/tools/res_timeline.py --model shipped --form one --out $R/gpurun_out/lat/tl_one.json > $R/gpurun_out/lat/tl.log 2>&1 || { tail -20 $R/gpurun_out/lat/tl.log; exit 1; }
cat $R/gpurun_out/lat/tl_one.json
