/* capi_smoke.c — a compiled C caller of include/avr.h (the boundary pbrt's
 * Integrator::Create("volpath_mi355x") adapter binds: cpu/integrators.cpp:3658-3709).
 *
 * Renders the S-uniform absorber (GridMedium 8^3 of ones on [0,1]^3, sigma_a 1, sigma_s 0,
 * uniform infinite light Le 1, orthographic camera down +z) through
 *   avr_context_create -> avr_medium_grid -> avr_lights -> avr_camera -> avr_film ->
 *   avr_render -> avr_film_read / avr_last_pass_samples
 * and checks Beer-Lambert: the mean sample radiance of the interior pixels equals
 * exp(-(1 - 0.25/n)) (the half-voxel trilinear shell, containers.h:822-835) within 4 sigma,
 * and every pixel's filter-weight sum equals spp (box filter weight 1).
 * Exit status 0 = pass. Built by tests/test_capi_abi.py (compile + link, no GPU) and run by
 * tests/test_gpu_capi_caller.py on an MI355X. */
#include "avr.h"

#include <math.h>
#include <stdio.h>
#include <stdlib.h>

#define CHECK(call)                                                                \
    do {                                                                           \
        int rc_ = (call);                                                          \
        if (rc_ != AVR_OK) {                                                       \
            fprintf(stderr, "%s failed (%d): %s\n", #call, rc_, avr_last_error()); \
            return 2;                                                              \
        }                                                                          \
    } while (0)

int main(int argc, char **argv) {
    const int n = 8, W = 16, H = 16, spp = 256;
    int device = argc > 1 ? atoi(argv[1]) : 0;
    static float density[8 * 8 * 8], sigma_a[AVR_TABLE_SIZE], sigma_s[AVR_TABLE_SIZE], Lsky[AVR_TABLE_SIZE];
    static float sensor[3 * AVR_TABLE_SIZE];
    for (int i = 0; i < n * n * n; ++i) density[i] = 1.0f;
    for (int i = 0; i < AVR_TABLE_SIZE; ++i) {
        sigma_a[i] = 1.0f;
        sigma_s[i] = 0.0f;
        Lsky[i] = 1.0f;
    }
    for (int i = 0; i < 3 * AVR_TABLE_SIZE; ++i) sensor[i] = 1.0f;
    const float bounds[6] = {0, 0, 0, 1, 1, 1};
    const float eye[16] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1};
    const int mres[3] = {16, 16, 16};
    /* OrthographicCamera, screen window [-0.5, 0.5]^2: raster (x, y) -> camera
     * (x/W - 0.5, 0.5 - y/H, 0); camera at (0.5, 0.5, -1) looking down +z */
    const float cam_from_raster[16] = {1.0f / W, 0, 0, -0.5f, 0, -1.0f / H, 0, 0.5f, 0, 0, 1, 0, 0, 0, 0, 1};
    const float render_from_cam[16] = {1, 0, 0, 0.5f, 0, 1, 0, 0.5f, 0, 0, 1, -1, 0, 0, 0, 1};
    const int light_type = 1;
    const float w3[3] = {0, 0, 1}, light_scale = 1.0f;
    const float radius[2] = {0.5f, 0.5f};

    avr_context *ctx = NULL;
    CHECK(avr_context_create(device, 0, &ctx));
    CHECK(avr_medium_grid(ctx, density, n, n, n, bounds, eye, eye, sigma_a, sigma_s, 0.0f, NULL, NULL, 0, 0, 0, mres));
    CHECK(avr_lights(ctx, 1, &light_type, w3, Lsky, &light_scale, 0.8660254f));
    CHECK(avr_camera(ctx, 0, cam_from_raster, render_from_cam));
    CHECK(avr_film(ctx, W, H, radius, sensor, 1.0f, 1e30f));
    CHECK(avr_set_sampler(ctx, 0, spp));
    CHECK(avr_render(ctx, 0, spp, 0, 5));

    double *rgb = malloc(sizeof(double) * 3 * W * H), *wsum = malloc(sizeof(double) * W * H);
    float *L = malloc(sizeof(float) * 4 * W * H * spp), *lam = malloc(sizeof(float) * 4 * W * H * spp),
          *pdf = malloc(sizeof(float) * 4 * W * H * spp);
    int first = -1, ns = 0;
    CHECK(avr_film_read(ctx, rgb, wsum));
    CHECK(avr_last_pass_samples(ctx, L, lam, pdf, (long long)W * H * spp, &first, &ns));
    int bad = 0;
    for (int p = 0; p < W * H; ++p)
        if (wsum[p] != (double)spp) bad = 1;
    if (bad) fprintf(stderr, "filter weight sums differ from spp\n");
    /* radiance of the last pass's samples of the interior pixels (box crossing of length 1) */
    double sum = 0;
    long long cnt = 0;
    for (int s = 0; s < ns; ++s)
        for (int y = 2; y < H - 2; ++y)
            for (int x = 2; x < W - 2; ++x) {
                sum += L[4 * ((long long)s * W * H + y * W + x)];
                ++cnt;
            }
    const double mean = sum / (double)cnt, want = exp(-(1.0 - 0.25 / n));
    const double tol = 4 * sqrt(want * (1 - want) / (double)cnt);
    printf("capi_smoke: pass [%d, %d), %lld interior samples, mean L %.5f, Beer-Lambert %.5f (tol %.5f)\n", first,
           first + ns, cnt, mean, want, tol);
    if (fabs(mean - want) > tol) bad = 1;
    CHECK(avr_context_destroy(ctx));
    free(rgb);
    free(wsum);
    free(L);
    free(lam);
    free(pdf);
    return bad;
}
