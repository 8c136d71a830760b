#!/bin/bash
# Round-3 GPU pass: GPU parity tests, the default bench line, and the N=2
# rehearsal through bench.py's own rank launcher (two ranks on cuda:0, gloo).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r03
mkdir -p $O
timeout -k 10 700 python3 -u -m pytest tests/ -m gpu -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo "gpu tests failed"; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python3 $R/bench.py --steps 1000 > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
timeout -k 10 200 python3 $R/bench.py --gpus 2 --same-device --dist-backend gloo --steps 200 --no-cpu --no-latency --no-ctl --no-gru > $O/bench_n2.json 2> $O/bench_n2.err || { echo "n2 failed"; tail -20 $O/bench_n2.err; exit 1; }
cat $O/bench_n2.json
timeout -k 10 200 python3 $R/bench.py --workload go2_gru_256_b4096_seq100 --steps 30 --warmup 2 --no-cpu --no-latency --no-ctl > $O/bench_gru_seq.json 2> $O/bench_gru_seq.err || { echo "gru seq failed"; tail -20 $O/bench_gru_seq.err; exit 1; }
cat $O/bench_gru_seq.json
