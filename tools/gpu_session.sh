# one GPU call of round 3's experiments (bash tools/gpu_session.sh on the box)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
RS_SPC=0 timeout -k 10 300 python -u tools/rank_share.py > gpurun_out/rank_share_r03e.txt 2>&1 || exit $?
bash tools/round_check.sh r03e || exit $?
