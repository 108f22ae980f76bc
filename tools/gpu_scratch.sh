set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_multi.py tests/test_gpu_benched_path.py tests/test_reference_binding.py -m gpu -v -s --timeout 200 --timeout-method thread > gpurun_out/new_tests.log 2>&1 || exit $?
AB_SPP=256 AB_ROUNDS=3 AB_SPC=0 AB_SCENES=random_ned timeout -k 10 300 python -u tools/ab.py ray-tracing-one-weekend_amd/librtow_hip.so ab/reorder/pkg/librtow_hip.so > gpurun_out/ab_reorder.txt 2>&1 || exit $?
