set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests/test_gpu_parity.py -q > gpurun_out/t3.log 2>&1; echo "pytest rc=$?"; tail -3 gpurun_out/t3.log
for w in 4 8; do timeout -k 10 300 python bench.py --waves $w --no-cpu --no-latency > gpurun_out/b_w$w.json 2>gpurun_out/b_w$w.err; echo "bench w$w rc=$?"; cat gpurun_out/b_w$w.json; done
bash tools/profile.sh
find gpurun_out/prof_mlp_kt -name '*.csv' | head; 
