set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/round_check.sh r05 configs,validate || exit $?
RS_SCENE=final_ned RS_WORLDS=8 RS_CHECK=1000 timeout -k 10 400 python -u tools/rank_share.py > gpurun_out/rank_share_final_ned_r05.txt 2>&1 || exit $?
