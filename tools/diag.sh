#!/bin/bash
# Diagnostics for the batched kernel (GPU box, repo root): ablation timings and PMC counters.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out/diag
W=${W:-8}
for v in noload nomfma; do
  GO2PI_LIB=$R/go2_onnx_controller_amd/lib/diag/libgo2pi_$v.so timeout -k 10 120 python3 $R/bench.py --waves $W --no-cpu --no-latency > $R/gpurun_out/diag/b_$v.json 2>&1 || exit 1
  python3 -c "import json;d=json.load(open('$R/gpurun_out/diag/b_$v.json'));print('$v', d['kernel_us'])"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 60 rocprofv3 -L > $R/gpurun_out/diag/counters.txt 2>&1
i=0
for set in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE" \
           "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SALU SQ_VALU_MFMA_BUSY_CYCLES" \
           "TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum" "TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum" \
           "SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $set --kernel-trace --output-format csv -d $R/gpurun_out/diag/pmc$i -o run -- python3 $R/bench.py --waves $W --steps 20 --warmup 5 --no-cpu --no-latency > $R/gpurun_out/diag/pmc$i.log 2>&1
  echo "pmc pass $i rc=$?"
done
exit 0
