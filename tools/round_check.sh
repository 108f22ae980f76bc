#!/bin/bash
# One GPU call: the bench kernel's profile (tools/profile_bench.sh TAG), the
# GPU test suite, smoke(), and every BASELINE config at full size
# (tools/bench_configs.py).  GPU box, repo root: bash tools/round_check.sh TAG
set -o pipefail
TAG=${1:-r02}
R=$(pwd)
mkdir -p gpurun_out
bash tools/profile_bench.sh $TAG > gpurun_out/profile_$TAG.log 2>&1 || exit $?
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread \
    > gpurun_out/gputests_$TAG.log 2>&1 || exit $?
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || exit $?
timeout -k 10 600 python tools/bench_configs.py --configs 1,2,3,4,5 --cpu-seconds 3 \
    --out gpurun_out/configs_$TAG.jsonl > gpurun_out/configs_$TAG.log 2>&1
