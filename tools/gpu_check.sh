# GPU round trip used during development: parity tests, then bench per wave count.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests/ -m gpu -q -x > gpurun_out/tests.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/tests.log
[ $rc -eq 0 ] || exit 1
for w in ${WAVES:-4 8 16}; do timeout -k 10 300 python bench.py --waves $w --no-cpu --no-latency > gpurun_out/b_w$w.json 2>gpurun_out/b_w$w.err || exit 1; python3 -c "import json;d=json.load(open('gpurun_out/b_w$w.json'));print('w$w', d['value'], d['kernel_us'], d['roofline']['frac'])"; done
