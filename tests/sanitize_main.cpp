// Host-side sanitizer run (ASan/UBSan on the CPU side). Built by
// tests/test_sanitize.py with g++ -fsanitize=address,undefined -fno-sanitize-recover=all:
// one translation unit holding the CPU oracle (oracle/volpath_oracle.cpp, test
// infrastructure), the host FreeGraph builder (avr_graph_host.h, the C-ABI's host code) and the
// shared sampler header (avr_sampling.h). It renders small scenes through every oracle code
// path the tests use (box and sphere interfaces, Independent / ZSobol, box / Gaussian filter,
// maxdepth 0..100, 1x2 and 7x8 films, both libm modes, 64-bit ZSobol indices), ratio-tracks transmittance and merges random walks
// into a graph; any out-of-bounds access, use-after-free, leak or undefined behaviour aborts.
#include "../oracle/volpath_oracle.cpp"
#include "../acceleratedvolrenderer_amd/csrc/avr_graph_host.h"
#define AVR_HD inline
#include "../acceleratedvolrenderer_amd/csrc/avr_sampling.h"

#include <cstdio>
#include <cstring>
#include <random>
#include <vector>

static void identity(float *m) {
    std::memset(m, 0, 16 * sizeof(float));
    m[0] = m[5] = m[10] = m[15] = 1.f;
}

int main() {
    std::mt19937 gen(7);
    std::uniform_real_distribution<float> U(0.f, 1.f);
    const int n = 12;
    std::vector<float> density(n * n * n);
    for (auto &v : density) v = 0.2f + U(gen);
    std::vector<float> sa(471, 0.5f), ss(471, 2.f), le(471, 0.f), xyz(3 * 471), lL(2 * 471, 1.f), lescale(1, 1.f);
    for (int i = 0; i < 471; ++i) {
        xyz[i] = U(gen);
        xyz[471 + i] = 0.5f + U(gen);
        xyz[942 + i] = U(gen);
        sa[i] = 0.2f + 0.8f * i / 470.f;   // chromatic: the 4-wavelength path
    }
    std::vector<float> maj(16 * 16 * 16);
    oracle_build_majorant(density.data(), n, n, n, 16, 16, 16, maj.data());

    OracleScene s;
    std::memset(&s, 0, sizeof(s));
    s.density = density.data();
    s.nx = s.ny = s.nz = n;
    const float b[6] = {0, 0, 0, 1, 1, 1};
    std::memcpy(s.bounds, b, sizeof(b));
    identity(s.render_from_medium);
    identity(s.medium_from_render);
    s.sigma_a = sa.data();
    s.sigma_s = ss.data();
    s.g = 0.3f;
    s.Le = le.data();
    s.Lescale = lescale.data();
    s.lnx = s.lny = s.lnz = 1;
    s.majorant = maj.data();
    s.mres[0] = s.mres[1] = s.mres[2] = 16;
    s.nlights = 2;
    s.light_type[0] = 0;
    s.light_w[0][0] = 0.577f; s.light_w[0][1] = 0.577f; s.light_w[0][2] = -0.577f;
    s.light_type[1] = 1;
    s.light_L[0] = lL.data();
    s.light_L[1] = lL.data() + 471;
    s.light_scale[0] = 2.f;
    s.light_scale[1] = 0.25f;
    s.scene_radius = 0.87f;
    s.camera_type = 0;
    identity(s.camera_from_raster);
    identity(s.render_from_camera);
    s.render_from_camera[3] = 0.5f; s.render_from_camera[7] = 0.5f; s.render_from_camera[11] = -1.f;
    s.filter_radius[0] = s.filter_radius[1] = 0.5f;
    s.sensor_xyz = xyz.data();
    s.imaging_ratio = 1.f;
    const float o2s[9] = {3.2f, -1.5f, -0.5f, -1.f, 1.9f, 0.04f, 0.05f, -0.2f, 1.05f};
    std::memcpy(s.output_from_sensor, o2s, sizeof(o2s));
    s.max_component_value = 1e30f;
    s.max_depth = 5;
    s.samples_per_pixel = 64;
    s.filter_sigma = 0.5f;
    s.film_lambda_min = 360.f;
    s.film_lambda_max = 830.f;

    long long total = 0;
    for (int boundary = 0; boundary < 2; ++boundary)
        for (int sampler = 0; sampler < 2; ++sampler)
            for (int filter = 0; filter < 2; ++filter)
                for (int depth : {0, 1, 5, 100})
                    for (int res : {1, 7}) {
                        s.boundary = boundary;
                        s.sphere[0] = s.sphere[1] = s.sphere[2] = 0.5f;
                        s.sphere[3] = 0.45f;
                        s.sampler_type = sampler;
                        s.filter_type = filter;
                        s.filter_radius[0] = s.filter_radius[1] = filter ? 1.5f : 0.5f;
                        s.max_depth = depth;
                        s.width = res;
                        s.height = res + 1;
                        const float sx = 1.f / res, sy = -1.f / (res + 1);
                        s.camera_from_raster[0] = sx; s.camera_from_raster[3] = -0.5f;
                        s.camera_from_raster[5] = sy; s.camera_from_raster[7] = 0.5f;
                        std::vector<double> rgb(3 * res * (res + 1)), w(res * (res + 1));
                        for (int libm = 0; libm < 2; ++libm) {
                            oracle_set_libm(libm);
                            total += oracle_render(&s, 0, 3, 2, rgb.data(), w.data());
                        }
                    }
    oracle_set_libm(0);
    std::vector<float> p0(3 * 64), p1(3 * 64), lam(4 * 64), tr(4 * 64);
    for (int i = 0; i < 64; ++i) {
        for (int k = 0; k < 3; ++k) { p0[3 * i + k] = U(gen); p1[3 * i + k] = U(gen); }
        for (int k = 0; k < 4; ++k) lam[4 * i + k] = 400.f + 100.f * k;
    }
    oracle_transmittance4(&s, 64, p0.data(), p1.data(), lam.data(), tr.data());

    avr::graph::Builder g(0.05f);
    std::vector<float> pts(3 * 8);
    for (int w = 0; w < 200; ++w) {
        const int k = (int)(U(gen) * 8);
        for (auto &v : pts) v = U(gen);
        g.AddWalk(pts.data(), k, k == 7, w % 5 == 0 && g.NumVertices() ? (int)(U(gen) * g.NumVertices()) : -1);
    }
    avr::smp::ZSobolParams zp = avr::smp::zsobol_params(4096, 1920, 1080, 3);
    avr::smp::ZSobol z;
    z.start(1919, 1079, 4095, zp);
    float acc = 0;
    for (int d = 0; d < 40; ++d) acc += z.get1d(zp);
    std::printf("sanitize ok: %lld oracle events, %zu graph vertices, %zu edges, zsobol sum %.3f\n", total,
                g.NumVertices(), g.NumEdges(), acc);
    return 0;
}
