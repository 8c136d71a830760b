set -o pipefail
bash tools/gpu_tests.sh || exit 1
for w in go2_lstm_256_b4096 go2_lstm_256_b4096_seq100 go2_gru_256_b4096_seq100; do timeout -k 10 200 python3 bench.py --workload $w --steps 30 --warmup 3 --no-cpu --no-latency --no-ctl > gpurun_out/t/b_$w.json 2> gpurun_out/t/b_$w.err || { echo "bench $w failed"; tail gpurun_out/t/b_$w.err; exit 1; }; python3 -c "import json;d=json.load(open('gpurun_out/t/b_$w.json'));print('$w', d['kernel_us'], d['roofline']['frac'], d['value'])"; done
