#!/bin/bash
# One GPU call: the GPU test suite, smoke(), the bench kernel's profile and the
# general configs' profiles (tools/profile_bench.sh TAG_<workload>), and every
# BASELINE config at full size (tools/bench_configs.py), whole-frame parity of
# every config against the oracle (tools/validate.py).
# GPU box, repo root: bash tools/round_check.sh TAG [steps: tests,profile,general,configs,validate]
set -o pipefail
TAG=${1:-r03}
STEPS=${2:-tests,profile,general,configs,validate}
R=$(pwd)
mkdir -p gpurun_out
if [[ $STEPS == *tests* ]]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread \
      > gpurun_out/gputests_$TAG.log 2>&1 || exit $?
  timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || exit $?
fi
if [[ $STEPS == *profile* ]]; then
  bash tools/profile_bench.sh $TAG > gpurun_out/profile_$TAG.log 2>&1 || exit $?
fi
if [[ $STEPS == *general* ]]; then
  for w in cornell cornell_smoke; do
    bash tools/profile_bench.sh ${TAG}_$w --workload $w --cpu-pixels 16000 > gpurun_out/profile_${TAG}_$w.log 2>&1 || exit $?
  done
  # config 5 at its full 4096x4096 frame, 256 spp per launch (VALU per ray does not depend on spp)
  bash tools/profile_bench.sh ${TAG}_final_ned --workload final_ned --spp 256 --cpu-pixels 8000 --cpu-spp 512 \
      > gpurun_out/profile_${TAG}_final_ned.log 2>&1 || exit $?
fi
if [[ $STEPS == *configs* ]]; then
  cd $R
  timeout -k 10 600 python tools/bench_configs.py --configs 1,2,3,4,5 --cpu-seconds 3 \
      --out gpurun_out/configs_$TAG.jsonl > gpurun_out/configs_$TAG.log 2>&1 || exit $?
fi
if [[ $STEPS == *validate* ]]; then
  cd $R
  timeout -k 10 600 python tools/validate.py --out gpurun_out/validation_$TAG.jsonl > gpurun_out/validate_$TAG.log 2>&1 || exit $?
fi
