set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
AB_SPP=256 AB_ROUNDS=5 AB_SPC=0 AB_SCENES=final_ned timeout -k 10 300 python -u tools/ab.py ab/main/librtow_hip.so ab/gridq/librtow_hip.so ab/gridq_def/librtow_hip.so > gpurun_out/ab_gridq_r05.txt 2>&1 || exit $?
