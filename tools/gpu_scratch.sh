set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
AB_SPP=256 AB_ROUNDS=5 AB_SPC=0 AB_SCENES=cornell,cornell_smoke timeout -k 10 500 python -u tools/ab.py ab/u_minreg/librtow_hip.so ab/k2minreg/librtow_hip.so ab/k2mmc/librtow_hip.so ab/k5minreg/librtow_hip.so ab/k5mmc/librtow_hip.so > gpurun_out/ab_sched_r05.txt 2>&1 || exit $?
