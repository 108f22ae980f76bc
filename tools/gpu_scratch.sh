set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
AB_SPP=256 AB_ROUNDS=3 AB_SPC=0 AB_SCENES=cornell,cornell_smoke,final_ned timeout -k 10 500 python -u tools/ab.py ab/main/librtow_hip.so ab/topsph/librtow_hip.so > gpurun_out/ab_topsph_r05.txt 2>&1 || exit $?
