set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
AB_SPP=256 AB_ROUNDS=5 AB_SPC=0 AB_SCENES=random_ned timeout -k 10 300 python -u tools/ab.py ab/main/librtow_hip.so ab/s_minreg/librtow_hip.so ab/s_mmc/librtow_hip.so ab/s_maxilp/librtow_hip.so > gpurun_out/ab_simple_sched_r05.txt 2>&1 || exit $?
bash tools/round_check.sh r05 configs,validate || exit $?
RS_SCENE=final_ned RS_WORLDS=8 RS_CHECK=1000 timeout -k 10 400 python -u tools/rank_share.py > gpurun_out/rank_share_final_ned_r05.txt 2>&1 || exit $?
timeout -k 10 200 python -u tools/prof_counters.py final_ned 32 > gpurun_out/prof_counters_final_ned_r05.txt 2>&1 || exit $?
