set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
AB_SPP=256 AB_ROUNDS=3 AB_SPC=0 AB_SCENES=final_ned timeout -k 10 400 python -u tools/ab.py ab/base/librtow_hip.so ab/lds/librtow_hip.so ab/tail/librtow_hip.so ab/spec3/librtow_hip.so > gpurun_out/ab_grid2_r05.txt 2>&1 || exit $?
for v in tail spec3; do
RTOW_LIB=ab/$v/librtow_hip.so timeout -k 10 200 python -u tools/prof_counters.py final_ned 32 > gpurun_out/prof_final_ned_$v.txt 2>&1 || exit $?
done
