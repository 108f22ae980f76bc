/*
 * rtow_rng.h — the counter-based random stream that replaces the reference's
 * global std::mt19937_64 (rngs.h:9-11).
 *
 * The reference draws every random number from ONE engine shared by all render
 * threads, seeded from the wall clock (main.cpp:82-88), so it has no
 * reproducible output.  This header defines the stream all components agree on
 * instead ("seeded identically"):
 *
 *   - every draw is a 24-bit integer r24, and the uniform is U = r24 * 2^-24.
 *     A float represents U exactly, and libstdc++'s
 *     uniform_real_distribution<double>(0,1) over an engine that returns
 *     (r24 << 40) yields exactly the same double (generate_canonical makes one
 *     engine call for a 64-bit engine), which is how the oracle harness injects
 *     this stream into the unmodified reference headers.
 *   - a stream is a 64-bit key plus a 32-bit draw counter; draw n of stream k is
 *     rtow_draw24(k, n).  Nothing is stateful besides the counter, so a GPU lane
 *     and a CPU thread produce the same numbers for the same (key, counter).
 *   - render streams are keyed per (seed, pixel, sample): the pixel index is
 *     row * W + column with the reference's row numbering (row 0 = bottom image
 *     row, main.cpp:932), so results do not depend on how pixels are split
 *     across threads, waves or GPUs.  The counter restarts at 0 for each sample
 *     and advances in the reference's draw order (jitter u, jitter v, camera
 *     time, then traversal / scatter draws).
 *   - the scene stream (Perlin tables at static init, noise.h:112-116, then the
 *     scene builder's draws, scenes.h:159-180, and one draw per BvhNode,
 *     bvhNode.h:26) is rtow_scene_key(scene_seed), counter from 0.
 *
 * Plain C99 so the C oracle can include it; under C++ the functions are
 * constexpr, which the HIP compiler also makes available in device code.
 */
#ifndef RTOW_RNG_H
#define RTOW_RNG_H

#include <stdint.h>

#ifdef __cplusplus
#define RTOW_RNG_FN constexpr inline
#else
#define RTOW_RNG_FN static inline
#endif

/* Wellons' "lowbias32" integer finaliser: a bijection on 32 bits. */
RTOW_RNG_FN uint32_t rtow_lowbias32(uint32_t x) {
    x ^= x >> 16;
    x *= 0x7feb352dU;
    x ^= x >> 15;
    x *= 0x846ca68bU;
    x ^= x >> 16;
    return x;
}

/* splitmix64 finaliser: a bijection on 64 bits, used only to derive keys. */
RTOW_RNG_FN uint64_t rtow_mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
    return z ^ (z >> 31);
}

/* Key of the render stream of one (pixel, sample). */
RTOW_RNG_FN uint64_t rtow_sample_key(uint64_t seed, uint32_t pixel, uint32_t sample) {
    return rtow_mix64(seed ^ rtow_mix64(((uint64_t)pixel << 32) | (uint64_t)sample));
}

/* Key of the scene-construction stream. */
RTOW_RNG_FN uint64_t rtow_scene_key(uint64_t scene_seed) {
    return rtow_mix64(scene_seed + 0x9E3779B97F4A7C15ULL);
}

/* Draw n of stream `key`: a 24-bit integer. */
RTOW_RNG_FN uint32_t rtow_draw24(uint64_t key, uint32_t n) {
    return rtow_lowbias32(rtow_lowbias32(n ^ (uint32_t)key) + (uint32_t)(key >> 32)) >> 8;
}

/* The uniform in [0,1) that draw n stands for (exact in float and double). */
RTOW_RNG_FN float rtow_draw_unit(uint64_t key, uint32_t n) {
    return (float)rtow_draw24(key, n) * (1.0f / 16777216.0f);
}

#endif /* RTOW_RNG_H */
