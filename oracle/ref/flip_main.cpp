// Test infrastructure: runs the reference's vendored FLIP (src/ext/flip/flip.cpp, compiled
// unmodified from /root/reference by oracle/ref/Makefile) on raw float RGB images.
// usage: flip_ref <test.f32> <ref.f32> <width> <height> <ppd> <out.f32>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "ext/flip/flip.h"

int main(int argc, char **argv) {
    if (argc != 7) {
        fprintf(stderr, "usage: flip_ref test.f32 ref.f32 width height ppd out.f32\n");
        return 2;
    }
    const int w = atoi(argv[3]), h = atoi(argv[4]);
    const float ppd = (float)atof(argv[5]);
    std::vector<float> test(3 * (size_t)w * h), ref(3 * (size_t)w * h), out((size_t)w * h);
    FILE *f = fopen(argv[1], "rb");
    if (!f || fread(test.data(), 4, test.size(), f) != test.size()) return 1;
    fclose(f);
    f = fopen(argv[2], "rb");
    if (!f || fread(ref.data(), 4, ref.size(), f) != ref.size()) return 1;
    fclose(f);
    FLIPOptions opt;
    opt.ppd = ppd;
    ComputeFLIPError(test.data(), ref.data(), out.data(), w, h, opt);
    f = fopen(argv[6], "wb");
    fwrite(out.data(), 4, out.size(), f);
    fclose(f);
    return 0;
}
