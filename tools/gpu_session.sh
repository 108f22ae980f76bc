# one GPU call of round 4 (bash tools/gpu_session.sh on the box): the GPU suite
# (benched-path parity, rtow_multi, the tiny-direction sqrt ray included),
# A/Bs -- scalar scene loads vs round 3's build on the general scenes; on
# config 2 the per-ray exact/fast sqrt switch (new) vs the build before it
# (cur), and the 4-wide tree (RTOW_WIDE=3/4) -- the instrumented bench
# kernel's counters, and config 5's eight rank shares at full size with the
# assembled frame checked against the oracle
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread \
    > gpurun_out/gputests_r04a.log 2>&1 || exit $?
AB_SPP=256 AB_ROUNDS=3 AB_SPC=0 AB_SCENES=cornell,cornell_smoke,final_ned timeout -k 10 300 \
    python -u tools/ab.py ab/base.so ab/new.so > gpurun_out/ab_scalar_r04a.txt 2>&1 || exit $?
AB_SPP=256 AB_ROUNDS=3 AB_SPC=0 AB_SCENES=random_ned timeout -k 10 300 \
    python -u tools/ab.py ab/base.so ab/cur.so ab/new.so ab/new.so:RTOW_WIDE=3 ab/new.so:RTOW_WIDE=4 ab/new.so:RTOW_WIDE=4,RTOW_SPEC=1 ab/new.so:RTOW_WIDE=4,RTOW_SPEC=24 \
    > gpurun_out/ab_wide_r04a.txt 2>&1 || exit $?
timeout -k 10 120 python -u tools/prof_counters.py random_ned 32 > gpurun_out/prof_r04a.txt 2>&1 || exit $?
RS_SCENE=final_ned RS_WORLDS=8 RS_CHECK=1000 timeout -k 10 600 python -u tools/rank_share.py \
    > gpurun_out/rank_share_final_r04a.txt 2>&1 || exit $?
