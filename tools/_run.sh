set -o pipefail
timeout -k 10 600 python -m pytest tests/ -m gpu -q -x > gpurun_out/tests.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/tests.log; [ $rc = 0 ] || { grep -E "^E |FAILED" gpurun_out/tests.log | head; exit 1; }
for w in 4 8 16; do timeout -k 10 300 python bench.py --workload go2_gru_256_b4096 --waves $w --no-cpu --no-latency 2>/dev/null | python3 -c "import json,sys;d=json.load(sys.stdin);print('gru w$w',d['value'],d['kernel_us'],d['roofline']['frac'])"; done
