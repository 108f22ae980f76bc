# one GPU call of round 3's experiments (bash tools/gpu_session.sh on the box)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 ./tools/sqrt_check > gpurun_out/sqrt_check.log 2>&1 || exit $?
bash tools/round_check.sh r03b tests,profile,general || exit $?
