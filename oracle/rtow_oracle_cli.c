/* rtow_oracle_cli.c — TEST INFRASTRUCTURE ONLY: command-line front end of the
 * C oracle (rtow_oracle.h), used to cross-check it against the reference
 * harness and to time the CPU baseline by hand.
 *   rtow_oracle <scene.scn> <camera.cam> <W> <H> <spp> <out_prefix> [seed] [threads]
 * writes <out_prefix>.lin / .bgra like oracle/_ref/ref_harness and prints the
 * traversal counters. */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include "rtow_oracle.h"

int main(int argc, char** argv) {
    if (argc < 7) {
        fprintf(stderr, "usage: rtow_oracle scene.scn camera.cam W H spp out_prefix [seed] [threads]\n");
        return 2;
    }
    rtow_oracle_scene* sc = NULL;
    if (rtow_oracle_load(argv[1], &sc)) { fprintf(stderr, "cannot load %s\n", argv[1]); return 2; }
    rtow_camera cam;
    FILE* f = fopen(argv[2], "rb");
    if (!f || fread(&cam, sizeof cam, 1, f) != 1) { fprintf(stderr, "cannot load %s\n", argv[2]); return 2; }
    fclose(f);
    rtow_params p;
    memset(&p, 0, sizeof p);
    p.width = (uint32_t)atoi(argv[3]);
    p.height = (uint32_t)atoi(argv[4]);
    p.spp = (uint32_t)atoi(argv[5]);
    p.max_depth = 50;
    p.gi_enable = 1;
    p.sky_gain = 1.0f;
    p.gi_gain = 0.3f;
    p.seed = argc > 7 ? strtoull(argv[7], NULL, 0) : 1;
    int threads = argc > 8 ? atoi(argv[8]) : 8;
    size_t npx = (size_t)p.width * p.height;
    float* lin = (float*)malloc(npx * 12);
    unsigned char* bgra = (unsigned char*)malloc(npx * 4);
    rtow_oracle_counters c;
    int rc = rtow_oracle_render(rtow_oracle_view(sc), &cam, &p, threads, lin, bgra, &c);
    if (rc) { fprintf(stderr, "render failed %d\n", rc); return 1; }
    char path[4096];
    snprintf(path, sizeof path, "%s.lin", argv[6]);
    f = fopen(path, "wb"); fwrite(lin, 4, npx * 3, f); fclose(f);
    snprintf(path, sizeof path, "%s.bgra", argv[6]);
    f = fopen(path, "wb"); fwrite(bgra, 1, npx * 4, f); fclose(f);
    printf("samples %llu segments %llu bvh_visits %llu bvh_pass %llu sphere %llu moving %llu rect %llu medium %llu draws %llu max_draws %llu\n",
           (unsigned long long)c.samples, (unsigned long long)c.segments, (unsigned long long)c.bvh_visits,
           (unsigned long long)c.bvh_box_pass, (unsigned long long)c.sphere_tests,
           (unsigned long long)c.moving_sphere_tests, (unsigned long long)c.rect_tests,
           (unsigned long long)c.medium_calls, (unsigned long long)c.draws,
           (unsigned long long)c.max_draws_per_sample);
    rtow_oracle_free(sc);
    free(lin);
    free(bgra);
    return 0;
}
