// Image-side kernels of the C-ABI (not on the path): RGBFilm::GetImage, the imgtool metrics and
// FLIP. Included by avr_kernels.hip after the path kernels (same translation unit, the C-ABI's).
#pragma once

namespace avr {

// RGBFilm::GetImage on the device (film.cpp:533-565): GetPixelRGB (film.h:258-274; rgbSum and
// weightSum rounded to float, divided, outputRGBFromSensorRGB applied as Mul's
// ((0 + m0 r) + m1 g) + m2 b; no splats) and, for the fp16 image, the 65504 clamp and the
// round-to-nearest-even half conversion.
struct Mat3 { float m[9]; };
__global__ void __launch_bounds__(256) k_film_image(DevFilm F, Mat3 M, int fp16, float *__restrict__ out) {
    const int np = F.width * F.height;
    for (int p = blockIdx.x * blockDim.x + threadIdx.x; p < np; p += gridDim.x * blockDim.x) {
        float r = (float)F.rgb_sum[3 * p], g = (float)F.rgb_sum[3 * p + 1], b = (float)F.rgb_sum[3 * p + 2];
        const float w = (float)F.w_sum[p];
        if (w != 0) { r /= w; g /= w; b /= w; }
        float o[3];
        for (int i = 0; i < 3; ++i) o[i] = (M.m[3 * i] * r + M.m[3 * i + 1] * g) + M.m[3 * i + 2] * b;
        if (fp16) {
            const float mx = fmaxf_(o[0], fmaxf_(o[1], o[2]));
            for (int i = 0; i < 3; ++i) {
                if (mx > 65504.f && o[i] > 65504.f) o[i] = 65504.f;
                o[i] = (float)(_Float16)o[i];   // IEEE round-to-nearest-even
            }
        }
        out[3 * p] = o[0];
        out[3 * p + 1] = o[1];
        out[3 * p + 2] = o[2];
    }
}

// Image::ME / MAE / MSE / MRSE terms (util/image.cpp:543-678) summed in f64: per thread over a
// grid-strided pixel range, then a fixed-order tree per block (deterministic for a fixed
// grid); k_metric_final adds the block partials in order. Slots per channel c: [c] for
// MAE/MSE/MRSE; ME: [c] absolute, [3 + c] positive, [6 + c] negative. Infinite terms skipped.
constexpr int kMetricSlots = 9;
__global__ void __launch_bounds__(256) k_metric(const float *__restrict__ img, const float *__restrict__ ref, int np,
                                                int metric, double *__restrict__ partial) {
    double acc[kMetricSlots];
    for (int k = 0; k < kMetricSlots; ++k) acc[k] = 0;
    for (int p = blockIdx.x * blockDim.x + threadIdx.x; p < np; p += gridDim.x * blockDim.x) {
        for (int c = 0; c < 3; ++c) {
            const double v = img[3 * p + c], vr = ref[3 * p + c];
            const double d = v - vr;
            double t;
            if (metric == 0) t = d * d;
            else if (metric == 1) t = d < 0 ? -d : d;
            else if (metric == 2) { const double q = vr + 0.01; t = (d * d) / (q * q); }
            else t = d;
            if (__builtin_isinf(t)) continue;
            if (metric == 3) {
                acc[c] += d < 0 ? -d : d;
                if (d > 0) acc[3 + c] += d;
                else acc[6 + c] += d;
            } else {
                acc[c] += t;
            }
        }
    }
    __shared__ double red[256];
    for (int k = 0; k < kMetricSlots; ++k) {
        red[threadIdx.x] = acc[k];
        __syncthreads();
        for (int s = blockDim.x / 2; s > 0; s >>= 1) {
            if ((int)threadIdx.x < s) red[threadIdx.x] += red[threadIdx.x + s];
            __syncthreads();
        }
        if (threadIdx.x == 0) partial[blockIdx.x * kMetricSlots + k] = red[0];
        __syncthreads();
    }
}
__global__ void k_metric_final(const double *__restrict__ partial, int nblocks, double *__restrict__ out) {
    const int k = threadIdx.x;
    if (k >= kMetricSlots) return;
    double s = 0;
    for (int b = 0; b < nblocks; ++b) s += partial[b * kMetricSlots + k];
    out[k] = s;
}

// FLIP (src/ext/flip/flip.cpp:941-984) — k_flip_prep: both images to YCxCz, w = the achromatic
// channel (Y + 16) / 116 the feature detectors read; k_flip_error: per pixel, the CSF
// convolution of both images (taps in the reference's row-major order, borders replicated),
// Lab + Hunt, HyAB colour difference, edge / point detector responses, error = cdiff^(1-fdiff).
__global__ void __launch_bounds__(256) k_flip_prep(const float *__restrict__ test, const float *__restrict__ ref, int n,
                                                   flip::F4 *__restrict__ ycT, flip::F4 *__restrict__ ycR) {
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        ycT[i] = flip::prep_pixel(test[3 * i], test[3 * i + 1], test[3 * i + 2]);
        ycR[i] = flip::prep_pixel(ref[3 * i], ref[3 * i + 1], ref[3 * i + 2]);
    }
}
__global__ void __launch_bounds__(256) k_flip_error(const flip::F4 *__restrict__ ycT, const flip::F4 *__restrict__ ycR,
                                                    int w, int h, const float *__restrict__ sf, int rs,
                                                    const float *__restrict__ ef, const float *__restrict__ pf, int rd,
                                                    float cmax, float *__restrict__ out) {
    const int n = w * h;
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x)
        out[i] = flip::error_at(ycT, ycR, w, h, i % w, i / w, sf, rs, ef, pf, rd, cmax);
}

}  // namespace avr
