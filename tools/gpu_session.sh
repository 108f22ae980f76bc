# one GPU call of round 3's experiments (bash tools/gpu_session.sh on the box)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k deep -v -s --timeout 200 --timeout-method thread > gpurun_out/deep_r03.log 2>&1 || exit $?
