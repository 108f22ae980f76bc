# Scratch GPU session (one gpurun call): the tests named in $GS_TESTS verbose
# (default: the round's new ones), then the whole GPU suite, then the bench
# (default path and --inproc).  Round-end profiles and configs:
# tools/round_check.sh.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${GS_TESTS:-tests/test_gpu_multi.py tests/test_gpu_benched_path.py tests/test_reference_binding.py}
timeout -k 10 400 python -u -m pytest $T -m gpu -v -s --timeout 200 --timeout-method thread \
    > gpurun_out/new_tests.log 2>&1 || exit $?
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
    > gpurun_out/gputests.log 2>&1 || exit $?
[ -n "$GS_NO_BENCH" ] && exit 0
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 > gpurun_out/bench.json 2> gpurun_out/bench.err || exit $?
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --inproc --no-cpu > gpurun_out/bench_inproc.json \
    2> gpurun_out/bench_inproc.err || exit $?
