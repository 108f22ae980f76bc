# one GPU call of round 4 (bash tools/gpu_session.sh on the box): A/B of the
# per-ray exact/fast sqrt switch on config 2 (new) vs the build before it
# (cur) and round 3's (base), the instrumented bench kernel's counters,
# config 5's eight rank shares at full size with the assembled frame checked
# against the oracle, then the 4-wide tree variants on small frames first
# (tools/wide_smoke.py; every traversal has a step bound that fails loudly)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_benched_path.py tests/test_gpu_sqrt.py tests/test_gpu_multi.py \
    -m gpu -v -s --timeout 240 --timeout-method thread > gpurun_out/gputests_numbers_r04b.log 2>&1 || exit $?
AB_SPP=256 AB_ROUNDS=3 AB_SPC=0 AB_SCENES=random_ned timeout -k 10 200 \
    python -u tools/ab.py ab/base.so ab/cur.so ab/new.so > gpurun_out/ab_sqrt_r04b.txt 2>&1 || exit $?
timeout -k 10 120 python -u tools/prof_counters.py random_ned 32 > gpurun_out/prof_r04b.txt 2>&1 || exit $?
RS_SCENE=final_ned RS_WORLDS=8 RS_CHECK=1000 timeout -k 10 600 python -u tools/rank_share.py \
    > gpurun_out/rank_share_final_r04b.txt 2>&1 || exit $?
timeout -k 10 150 python -u tools/wide_smoke.py 4 3 4:1 4:24 > gpurun_out/wide_smoke_r04b.txt 2>&1 || exit $?
