set -o pipefail
timeout -k 10 900 python -m pytest tests/ -m gpu -q > gpurun_out/tests.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/tests.log
grep -E "^FAILED|Error" gpurun_out/tests.log | head -20
