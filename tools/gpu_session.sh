# one GPU call of round 3's experiments (bash tools/gpu_session.sh on the box)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/gputests_r03d.log 2>&1
timeout -k 10 120 python tools/tie_measure.py > gpurun_out/tie_measure.log 2>&1 || exit $?
AB_SCENES=random_ned AB_SPP=1024 AB_ROUNDS=2 AB_SPC=0 timeout -k 10 300 python tools/ab.py ray-tracing-one-weekend_amd/librtow_hip.so ray-tracing-one-weekend_amd/librtow_hip.so:RTOW_AUTO_SPC=128 > gpurun_out/ab_spc128.log 2>&1 || exit $?
cd /tmp
RTOW_AUTO_SPC=128 timeout -k 10 -s KILL 200 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/pmc_spc128 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 1 --warmup 0 --no-cpu > $GRAFT_REPO_ROOT/gpurun_out/pmc_spc128.log 2>&1 || exit $?
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python bench.py > gpurun_out/bench_r03d.json 2> gpurun_out/bench_r03d.err
