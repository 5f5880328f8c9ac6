/* sanitize_oracle.c — drives the C restatement (oracle/sm_oracle.c, sm_oracle_agg.c; test
 * infrastructure) through every pipeline it implements on small synthetic pairs, for a build with
 * -fsanitize=address,undefined (tests/test_sanitizers.py): every cost method, CBCA / GF (both
 * forms) / NL / no aggregation, WTA / 4- and 8-path SGM / "so", Do_refine, the pyramid with PY_LVL
 * 2 and 3, shapes from 2 x 2 up, D above the width, and the bad-t evaluator.  Prints a checksum
 * of every map and "ok <runs>"; any sanitizer finding aborts the process. */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "sm_oracle.h"

static uint32_t rng_state = 12345u;
static uint32_t rnd(void) {
    rng_state = rng_state * 1664525u + 1013904223u;
    return rng_state >> 8;
}

/* a textured left image and the right image shifted by a per-row disparity ramp */
static void make_pair(int H, int W, int dmax, uint8_t* bl, uint8_t* br, uint8_t* gl, uint8_t* gr) {
    for (int i = 0; i < H * W * 3; i++) bl[i] = (uint8_t)(rnd() & 0xff);
    for (int y = 0; y < H; y++)
        for (int x = 0; x < W; x++) {
            const int d = dmax > 0 ? (y * 3 + x / 4) % (dmax + 1) : 0;
            const int xs = x + d < W ? x + d : W - 1;
            for (int c = 0; c < 3; c++) br[(y * W + x) * 3 + c] = bl[(y * W + xs) * 3 + c];
        }
    for (int i = 0; i < H * W; i++) {
        gl[i] = (uint8_t)((bl[3 * i] + 2 * bl[3 * i + 1] + bl[3 * i + 2]) / 4);
        gr[i] = (uint8_t)((br[3 * i] + 2 * br[3 * i + 1] + br[3 * i + 2]) / 4);
    }
}

static uint64_t checksum(const int16_t* d, int n) {
    uint64_t h = 1469598103934665603ull;
    for (int i = 0; i < n; i++) h = (h ^ (uint16_t)d[i]) * 1099511628211ull;
    return h;
}

int main(void) {
    setvbuf(stdout, NULL, _IONBF, 0);
    static const int shapes[][3] = {{2, 2, 1}, {3, 70, 9}, {24, 31, 15}, {40, 48, 40}, {17, 9, 20}};
    int runs = 0;
    for (size_t s = 0; s < sizeof shapes / sizeof shapes[0]; s++) {
        const int H = shapes[s][0], W = shapes[s][1], md = shapes[s][2];
        uint8_t* bl = malloc((size_t)H * W * 3);
        uint8_t* br = malloc((size_t)H * W * 3);
        uint8_t* gl = malloc((size_t)H * W);
        uint8_t* gr = malloc((size_t)H * W);
        int16_t* disp = malloc((size_t)H * W * sizeof(int16_t));
        float* gt = malloc((size_t)H * W * sizeof(float));
        uint8_t* mask = malloc((size_t)H * W);
        if (!bl || !br || !gl || !gr || !disp || !gt || !mask) return 2;
        make_pair(H, W, md, bl, br, gl, gr);
        for (int i = 0; i < H * W; i++) {
            gt[i] = (float)(rnd() % (unsigned)(md + 1));
            mask[i] = (uint8_t)((rnd() & 1) ? 255 : 0);
        }
        for (int cost = 0; cost < 4; cost++)
            for (int agg = 0; agg < 4; agg++)
                for (int opt = 0; opt < 3; opt++) {
                    /* NL needs rows, cols >= 3 (a spanning tree over the 4-neighbour grid) */
                    if (agg == 3 && (H < 3 || W < 3)) continue;
                    for (int variant = 0; variant < 2; variant++) {
                        /* the MY_GUIDE filter's box needs 2 r + 1 = 19 rows and columns */
                        if (agg == 2 && variant && (H < 19 || W < 19)) continue;
                        smo_config c;
                        smo_default_config(&c, md, H, W);
                        c.cost_method = cost;
                        c.aggregation = agg;
                        c.optimization = opt;
                        c.sgm_paths = variant ? 8 : 4;
                        c.do_refine = variant && opt != 0;
                        c.gf_mode = variant;
                        c.census_ring = (cost + agg) & 1;
                        if (smo_run(&c, bl, br, gl, gr, disp, NULL, NULL, NULL, NULL, NULL) != 0) {
                            printf("run failed: shape %zu cost %d agg %d opt %d variant %d\n", s, cost, agg, opt, variant);
                            return 1;
                        }
                        printf("%zu %d %d %d %d %016llx\n", s, cost, agg, opt, variant,
                               (unsigned long long)checksum(disp, H * W));
                        runs++;
                    }
                }
        {
            float rms = 0.f;
            const float bad = smo_bad_ratio(H, W, disp, gt, mask, 2.0f, &rms);
            printf("bad %zu %.6f %.6f\n", s, bad, rms);
        }
        for (int lvl = 2; lvl <= 3; lvl++) {
            if (H < 8 || W < 8) break;
            smo_config c;
            smo_default_config(&c, md, H, W);
            if (smo_run_pyr(&c, lvl, bl, br, gl, gr, disp) != 0) {
                printf("pyramid failed: shape %zu level %d\n", s, lvl);
                return 1;
            }
            printf("pyr %zu %d %016llx\n", s, lvl, (unsigned long long)checksum(disp, H * W));
            runs++;
        }
        free(bl);
        free(br);
        free(gl);
        free(gr);
        free(disp);
        free(gt);
        free(mask);
    }
    printf("ok %d\n", runs);
    return 0;
}
