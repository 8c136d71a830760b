set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests/ -m gpu -q -x > gpurun_out/tests.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/tests.log; [ $rc = 0 ] || { grep -E "^E |FAILED" gpurun_out/tests.log | head -20; exit 1; }
timeout -k 10 300 python bench.py > gpurun_out/b.json 2> gpurun_out/b.err || exit 1
cat gpurun_out/b.json
