set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_benched_path.py -x -v -s --timeout 300 --timeout-method thread > gpurun_out/benched_path_earth.txt 2>&1 || exit $?
timeout -k 10 300 python -u bench.py > gpurun_out/bench_earth.json 2> gpurun_out/bench_earth.err || exit $?
