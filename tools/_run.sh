set -o pipefail
timeout -k 10 300 python bench.py --no-cpu --no-latency > gpurun_out/b.json 2>gpurun_out/b.err || exit 1
python3 -c "import json;d=json.load(open('gpurun_out/b.json'));print(d['value'], d['kernel_us'], d['host_enqueue_us'], d['ms_per_step'], d['roofline']['frac'])"
TAG=w16 bash tools/profile.sh
python3 - <<'PY'
import csv
for r in csv.DictReader(open('gpurun_out/prof_w16_kt/run_kernel_stats.csv')): print(r['Name'][:60], r['Calls'], r['AverageNs'], r['MinNs'], r['MaxNs'])
PY
