/*
 * oracle_cli.c -- command-line front end of the CPU oracle (TEST INFRASTRUCTURE).
 *
 *   oracle_cli <scene.txt> <W> <H> <depth> [--threads N] [--p3 FILE] [--p6 FILE]
 *
 * Renders the full frame with the restatement in rt_oracle.c, prints one JSON
 * line {"primary":..,"shadow":..,"reflect":..,"seconds":..}.  Used to make the
 * golden fixtures (tests/golden/make_golden.py) and to cross-check the
 * reference build in oracle/_ref.
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "rt_oracle.h"

static double now_s(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + ts.tv_nsec * 1e-9;
}

int main(int argc, char **argv) {
    if (argc < 5) {
        fprintf(stderr, "usage: %s scene.txt W H depth [--threads N] [--p3 F] [--p6 F]\n", argv[0]);
        return 2;
    }
    const char *scene_path = argv[1];
    int W = atoi(argv[2]), H = atoi(argv[3]), D = atoi(argv[4]);
    int threads = 1;
    const char *p3 = NULL, *p6 = NULL;
    for (int i = 5; i < argc; i++) {
        if (!strcmp(argv[i], "--threads") && i + 1 < argc) threads = atoi(argv[++i]);
        else if (!strcmp(argv[i], "--p3") && i + 1 < argc) p3 = argv[++i];
        else if (!strcmp(argv[i], "--p6") && i + 1 < argc) p6 = argv[++i];
        else { fprintf(stderr, "unknown arg %s\n", argv[i]); return 2; }
    }
    orc_scene s;
    if (orc_load_scene(scene_path, &s, 0) != 0) {
        fprintf(stderr, "Could not open scene file: %s\n", scene_path);
        return 1;
    }
    uint8_t *rgb = (uint8_t *)malloc((size_t)W * H * 3);
    orc_counts c;
    double t0 = now_s();
    orc_render(&s, W, H, D, 1, 0, 1, H, rgb, NULL, &c, threads);
    double t1 = now_s();
    printf("{\"primary\": %llu, \"shadow\": %llu, \"reflect\": %llu, \"negative\": %llu, \"seconds\": %.6f, \"threads\": %d}\n",
           (unsigned long long)c.primary, (unsigned long long)c.shadow, (unsigned long long)c.reflect,
           (unsigned long long)c.negative, t1 - t0, threads);
    if (p3) orc_write_p3(p3, rgb, W, H);
    if (p6) {
        FILE *f = fopen(p6, "wb");
        fprintf(f, "P6\n%d %d\n255\n", W, H);
        fwrite(rgb, 1, (size_t)W * H * 3, f);
        fclose(f);
    }
    free(rgb);
    orc_free_scene(&s);
    return 0;
}
