set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_controller.py -q -x > gpurun_out/ctl.log 2>&1; rc=$?; echo "ctl pytest rc=$rc"; tail -3 gpurun_out/ctl.log; [ $rc = 0 ] || { grep -E "^E |FAILED|Error" gpurun_out/ctl.log | head -30; exit 1; }
timeout -k 10 900 python -m pytest tests/ -m gpu -q -x > gpurun_out/tests.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/tests.log; [ $rc = 0 ] || { grep -E "^E |FAILED" gpurun_out/tests.log | head; exit 1; }
