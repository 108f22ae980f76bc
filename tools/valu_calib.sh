#!/bin/bash
# Calibrates the SQ VALU counter pair on gfx950 (tools/valu_calib.hip): one
# PMC pass per active-lane count K, plus the host's CPU picture.
#   bash tools/valu_calib.sh   (GPU box, repo root; binary built in-tree)
set -o pipefail
R=$(pwd)
OUT=$R/gpurun_out/valu_calib
mkdir -p $OUT
export TMPDIR=/tmp
{ nproc; python3 -c 'import os; print(os.cpu_count(), len(os.sched_getaffinity(0)))';
  cat /sys/fs/cgroup/cpu.max 2>/dev/null; grep -m1 "model name" /proc/cpuinfo; } > $OUT/host.txt 2>&1
cd /tmp
for k in 64 32 16 1; do
  timeout -k 10 -s KILL 60 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAVE_CYCLES \
      SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE --kernel-trace -d $OUT/k$k -o run --output-format csv -- \
      $R/tools/valu_calib $k > $OUT/k$k.log 2>&1 || exit $?
done
echo calib done
