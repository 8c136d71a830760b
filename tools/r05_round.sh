#!/bin/bash
# r05 combined GPU pass: BAR probe, the GPU test suite, the batch-1 latency A/B
# (tools/r05_latency.sh), then the default bench line. Each step under its own
# time limit; a failing step ends the script.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
if [ -x $R/tools/bar_probe ]; then
  timeout -k 10 150 $R/tools/bar_probe > $O/bar.txt 2>&1; echo "bar_probe rc=$?"; cat $O/bar.txt
fi
timeout -k 10 1000 python3 -u -m pytest $R/tests -m gpu -x -q --timeout 120 --timeout-method thread ${SEL:-} > $O/tests.log 2>&1 || { echo "gpu tests failed"; grep -E "FAILED|ERROR|Error" $O/tests.log | head -20; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
[ -n "$NO_LAT" ] || bash $R/tools/r05_latency.sh > $O/lat.log 2>&1 || { echo "latency failed"; tail -20 $O/lat.log; exit 1; }
grep -E "round|p50" $O/lat/ab.txt | tail -18
timeout -k 10 600 python3 $R/bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
if [ -x $R/tools/launch_gap.bin ]; then
  timeout -k 10 120 $R/tools/launch_gap.bin > $O/launch_gap.txt 2>&1 || { echo "launch_gap failed"; cat $O/launch_gap.txt; exit 1; }
  cat $O/launch_gap.txt
fi
