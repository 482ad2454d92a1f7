// trt_bands.h — the interleaved row-band partition of a tiled frame (shared by the tracer's
// band launches, the multi-GPU exchange plan and the re-interleave kernel, host and device).
//
// Rows are dealt in bands of B rows to NG band groups: frame row y belongs to band b = y / B,
// group b % NG; group g's rows, in order, are its "compact" rows k = 0, 1, ...  (the
// reference renders every row on one GPU, main.cpp:2122-2124; SURVEY §8(e) spreads the costly
// image centre over every device this way).
#pragma once

#include <stdint.h>

#if defined(__HIPCC__) || defined(__HIP__)
#define TRT_HD __host__ __device__ __forceinline__
#else
#define TRT_HD inline
#endif

namespace trt {

// Frame row of compact row k of band group g (B rows per band, NG groups).
TRT_HD uint32_t band_frame_row(uint32_t k, uint32_t B, uint32_t NG, uint32_t g) {
    return ((k / B) * NG + g) * B + (k % B);
}

// Band group and compact row of frame row y.
TRT_HD void band_of_row(uint32_t y, uint32_t B, uint32_t NG, uint32_t& g, uint32_t& k) {
    const uint32_t b = y / B;
    g = b % NG;
    k = (b / NG) * B + y % B;
}

// Compact rows of band group g in a frame of H rows.
TRT_HD uint32_t band_group_rows(uint32_t H, uint32_t B, uint32_t NG, uint32_t g) {
    if (NG <= 1 || B == 0) return H;
    const uint32_t period = B * NG, full = H / period, rem = H % period;
    const uint32_t lo = g * B; // first row of the group within a period
    const uint32_t tail = rem > lo ? (rem - lo < B ? rem - lo : B) : 0u;
    return full * B + tail;
}

} // namespace trt
