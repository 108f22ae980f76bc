# one GPU call of round 3's experiments (bash tools/gpu_session.sh on the box)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/round_check.sh r03d || exit $?
