#!/bin/bash
# PMC passes over the trace kernel of the probe workload (one counter group
# per pass; --kernel-trace only beside --pmc).  Usage: bash tools/pmc_probe.sh TAG
set -o pipefail
TAG=${1:-cur}
R=$(pwd)
OUT=$R/gpurun_out/pmc_$TAG
mkdir -p $OUT
export TMPDIR=/tmp PROBE_WAVES=4 PROBE_ROUNDS=1 PROBE_ONLY=random_ned
cd /tmp
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU" \
           "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM" \
           "SQ_INST_LEVEL_VMEM SQ_INST_CYCLES_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_FLOPS_FP64 SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE" \
           "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $grp --kernel-trace -d $OUT/p$i -o run --output-format csv -- \
      python3 $R/tools/probe.py > $OUT/p$i.log 2>&1 || exit $?
done
python3 - "$OUT" <<'PY'
import csv, glob, json, sys
out = {}
for f in glob.glob(sys.argv[1] + "/p*/run_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        if "trace_kernel" in r["Kernel_Name"]:
            out[r["Counter_Name"]] = out.get(r["Counter_Name"], 0) + float(r["Counter_Value"])
json.dump(out, open(sys.argv[1] + "/summary.json", "w"), indent=1)
print(json.dumps(out, indent=1))
PY
