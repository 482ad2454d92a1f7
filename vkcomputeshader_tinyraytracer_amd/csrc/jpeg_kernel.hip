// jpeg_kernel.hip — GPU half of the envmap JPEG decoder: dequantisation,
// 8x8 integer IDCT, chroma upsampling and colour conversion, bit-exact with the kernels of the
// reference's stb_image v2.22 (lib/stb_image.h: stbi__idct_block / its SSE2 twin, the
// resample_row_* filters, stbi__YCbCr_to_RGB_row, stbi__blinn_8x8; load_jpeg_image).
//
// Layout: coefficients arrive as one int16 plane per component (blocks row-major, 64
// natural-order coefficients per block).  Kernel 1 works on 32 blocks per 256-thread
// workgroup, 8 lanes per block: each lane dequantises one 16-byte coefficient row, the
// column pass runs one column per lane through LDS, the row pass one row per lane, and every
// lane stores its 8 output samples as one 8-byte write into the component's sample plane.
// Kernel 2 is one thread per output pixel: it upsamples each component (the closed forms of
// stb's row filters, with the vertical near/far rows of its line-buffer walk precomputed on
// the host) and converts to RGBA8, one 4-byte store per pixel.  Both are HBM-bound streams
// (2 B in + 1 B out per sample, then ~1.5-3 B in + 4 B out per pixel).
#include <hip/hip_runtime.h>

#include <cstdint>
#include <vector>

#include "../../include/trt/abi.h"
#include "jpeg.h"

namespace trt {
namespace jpeg {

namespace {

// stb's fixed-point IDCT constants: (int)(x * 4096 + 0.5)
constexpr int fx(double x) { return (int)(x * 4096.0 + 0.5); }
constexpr int C0_5411961 = fx((double)0.5411961f), C_1_847759065 = fx((double)-1.847759065f);
constexpr int C0_765366865 = fx((double)0.765366865f), C1_175875602 = fx((double)1.175875602f);
constexpr int C0_298631336 = fx((double)0.298631336f), C2_053119869 = fx((double)2.053119869f);
constexpr int C3_072711026 = fx((double)3.072711026f), C1_501321110 = fx((double)1.501321110f);
constexpr int C_0_899976223 = fx((double)-0.899976223f), C_2_562915447 = fx((double)-2.562915447f);
constexpr int C_1_961570560 = fx((double)-1.961570560f), C_0_390180644 = fx((double)-0.390180644f);

// One 8-point pass of the islow (LLM) IDCT at 12 fractional bits.  On return
// o[k] = even[k] + odd[k] and o[7-k] = even[k] - odd[k] before the caller's bias and shift,
// i.e. the caller adds `bias` to the even terms then shifts.
__device__ __forceinline__ void idct8(const int s[8], int bias, int shift, int o[8]) {
    // even part: s0, s2, s4, s6
    const int e_rot = (s[2] + s[6]) * C0_5411961;
    const int e2 = e_rot + s[6] * C_1_847759065;
    const int e3 = e_rot + s[2] * C0_765366865;
    const int e0 = (s[0] + s[4]) * 4096;
    const int e1 = (s[0] - s[4]) * 4096;
    const int x0 = e0 + e3 + bias, x3 = e0 - e3 + bias;
    const int x1 = e1 + e2 + bias, x2 = e1 - e2 + bias;
    // odd part: s7, s5, s3, s1
    int a0 = s[7], a1 = s[5], a2 = s[3], a3 = s[1];
    const int q3 = a0 + a2, q4 = a1 + a3, q1 = a0 + a3, q2 = a1 + a2;
    const int q5 = (q3 + q4) * C1_175875602;
    a0 *= C0_298631336;
    a1 *= C2_053119869;
    a2 *= C3_072711026;
    a3 *= C1_501321110;
    const int r1 = q5 + q1 * C_0_899976223;
    const int r2 = q5 + q2 * C_2_562915447;
    const int r3 = q3 * C_1_961570560;
    const int r4 = q4 * C_0_390180644;
    a3 += r1 + r4;
    a2 += r2 + r3;
    a1 += r2 + r4;
    a0 += r1 + r3;
    o[0] = (x0 + a3) >> shift;
    o[7] = (x0 - a3) >> shift;
    o[1] = (x1 + a2) >> shift;
    o[6] = (x1 - a2) >> shift;
    o[2] = (x2 + a1) >> shift;
    o[5] = (x2 - a1) >> shift;
    o[3] = (x3 + a0) >> shift;
    o[4] = (x3 - a0) >> shift;
}

__device__ __forceinline__ uint32_t clamp8(int x) { return (uint32_t)min(max(x, 0), 255); }

// Opaque to the instruction selector.  Without it, hipcc (ROCm 7.2) fuses two
// clamp8(v >> n) into gfx950's v_ashr_pk_u8_i32 and ORs a third byte into bits 16-23 of that
// result, which the instruction does not leave zero: every third output byte came out
// corrupted (probe: tools/dbg/idct_probe.hip).
__device__ __forceinline__ int opaque(int x) {
    asm volatile("" : "+v"(x));
    return x;
}

constexpr int kBlocksPerGroup = 32; // 8 lanes per block, 256 threads

__global__ __launch_bounds__(256) void idct_kernel(const int16_t* __restrict__ coef,
                                                   const uint16_t* __restrict__ quant,
                                                   uint8_t* __restrict__ samples, uint32_t nblocks,
                                                   uint32_t bw, uint32_t stride) {
    __shared__ int tile[kBlocksPerGroup][8][9]; // [block][row][col], padded against conflicts
    const uint32_t lane = threadIdx.x & 7u, slot = threadIdx.x >> 3;
    const uint32_t blk = blockIdx.x * kBlocksPerGroup + slot;
    const bool live = blk < nblocks;
    if (live) { // dequantise row `lane`: (short)(coef * q), as stb's int16 multiply
        const uint4 raw = *reinterpret_cast<const uint4*>(coef + 64 * (size_t)blk + 8 * lane);
        const uint32_t w[4] = {raw.x, raw.y, raw.z, raw.w};
#pragma unroll
        for (int c = 0; c < 8; ++c) {
            const int16_t v = (int16_t)(c & 1 ? w[c >> 1] >> 16 : w[c >> 1] & 0xFFFFu);
            tile[slot][lane][c] = (int16_t)((int)v * (int)quant[8 * lane + c]);
        }
    }
    __syncthreads();
    if (live) { // columns: lane = column; keep 2 extra bits (>> 10 with rounding)
        int s[8], o[8];
#pragma unroll
        for (int r = 0; r < 8; ++r) s[r] = tile[slot][r][lane];
        idct8(s, 512, 10, o);
#pragma unroll
        for (int r = 0; r < 8; ++r) tile[slot][r][lane] = o[r];
    }
    __syncthreads();
    if (live) { // rows: lane = row; remove 1 << 17 with rounding, + 128 level shift, clamp
        int s[8], o[8];
#pragma unroll
        for (int c = 0; c < 8; ++c) s[c] = tile[slot][lane][c];
        idct8(s, 65536 + (128 << 17), 17, o);
#pragma unroll
        for (int c = 0; c < 8; ++c) o[c] = opaque(o[c]);
        const uint32_t lo = clamp8(o[0]) | clamp8(o[1]) << 8 | clamp8(o[2]) << 16 | clamp8(o[3]) << 24;
        const uint32_t hi = clamp8(o[4]) | clamp8(o[5]) << 8 | clamp8(o[6]) << 16 | clamp8(o[7]) << 24;
        const uint32_t bx = blk % bw, by = blk / bw;
        *reinterpret_cast<uint2*>(samples + (size_t)(8 * by + lane) * stride + 8 * bx) = make_uint2(lo, hi);
    }
}

enum Filter : int { F_COPY = 0, F_V2 = 1, F_H2 = 2, F_HV2 = 3, F_NEAREST = 4 };

struct CompArgs {
    const uint8_t* samples;
    const int32_t* rows; // per output row: near row, far row (sample-row indices)
    uint32_t stride;
    int filter, hs, w_lores;
};

struct ColorArgs {
    CompArgs c[4];
    uint32_t* out;
    int width, height, ncomp, color;
};

// One output sample of component a at pixel (x, y): the row filters of load_jpeg_image.
__device__ __forceinline__ int sample(const CompArgs& a, int x, int y) {
    const uint8_t* nr = a.samples + (size_t)a.rows[2 * y] * a.stride;
    const uint8_t* fr = a.samples + (size_t)a.rows[2 * y + 1] * a.stride;
    const int w = a.w_lores;
    switch (a.filter) {
    case F_COPY: return nr[x];
    case F_V2: return (3 * nr[x] + fr[x] + 2) >> 2;
    case F_H2: { // stbi__resample_row_h_2 (note its second-to-last output)
        if (w == 1 || x == 0) return nr[0];
        if (x == 2 * w - 1) return nr[w - 1];
        if (x == 2 * w - 2) return (3 * nr[w - 2] + nr[w - 1] + 2) >> 2;
        if (x == 1) return (3 * nr[0] + nr[1] + 2) >> 2;
        const int i = x >> 1;
        return (3 * nr[i] + 2 + ((x & 1) ? nr[i + 1] : nr[i - 1])) >> 2;
    }
    case F_HV2: { // stbi__resample_row_hv_2: t(i) = 3 near + far, then 3:1 across
        if (w == 1 || x == 0) return (3 * nr[0] + fr[0] + 2) >> 2;
        if (x == 2 * w - 1) return (3 * nr[w - 1] + fr[w - 1] + 2) >> 2;
        const int i = (x + 1) >> 1; // x = 2i - 1 (odd) or 2i (even), 1 <= i < w
        const int ta = 3 * nr[i - 1] + fr[i - 1], tb = 3 * nr[i] + fr[i];
        return (x & 1) ? (3 * ta + tb + 8) >> 4 : (3 * tb + ta + 8) >> 4;
    }
    default: return nr[x / a.hs]; // stbi__resample_row_generic (nearest)
    }
}

// stbi__float2fixed: ((int)(x * 4096.0f + 0.5f)) << 8
__device__ __forceinline__ constexpr int f2fix(float x) { return ((int)(x * 4096.0f + 0.5f)) * 256; }

__device__ __forceinline__ uint32_t ycbcr_to_rgba(int y, int cb, int cr) {
    const int32_t yf = (y << 20) + (1 << 19);
    cr -= 128;
    cb -= 128;
    const int32_t r = yf + cr * f2fix(1.40200f);
    // the Cb term of g is truncated to its top 16 bits, as stb's (reduced-precision) form
    const uint32_t cbg = (uint32_t)(cb * -f2fix(0.34414f)) & 0xFFFF0000u;
    const int32_t g = (int32_t)((uint32_t)yf + (uint32_t)(cr * -f2fix(0.71414f)) + cbg);
    const int32_t b = yf + cb * f2fix(1.77200f);
    return clamp8(opaque(r >> 20)) | clamp8(opaque(g >> 20)) << 8 | clamp8(opaque(b >> 20)) << 16 | 0xFF000000u;
}

__device__ __forceinline__ uint32_t blinn(uint32_t x, uint32_t m) { // stbi__blinn_8x8
    const uint32_t t = x * m + 128u;
    return ((t + (t >> 8)) >> 8) & 255u;
}

__global__ __launch_bounds__(256) void color_kernel(ColorArgs A) {
    const int x = (int)(blockIdx.x * 64 + (threadIdx.x & 63));
    const int y = (int)(blockIdx.y * 4 + (threadIdx.x >> 6));
    if (x >= A.width || y >= A.height) return;
    uint32_t px;
    if (A.color == TRT_JPEG_GRAY) {
        const uint32_t v = (uint32_t)sample(A.c[0], x, y);
        px = v | v << 8 | v << 16 | 0xFF000000u;
    } else if (A.color == TRT_JPEG_RGB) {
        px = (uint32_t)sample(A.c[0], x, y) | (uint32_t)sample(A.c[1], x, y) << 8 |
             (uint32_t)sample(A.c[2], x, y) << 16 | 0xFF000000u;
    } else if (A.color == TRT_JPEG_CMYK) {
        const uint32_t m = (uint32_t)sample(A.c[3], x, y);
        px = blinn((uint32_t)sample(A.c[0], x, y), m) | blinn((uint32_t)sample(A.c[1], x, y), m) << 8 |
             blinn((uint32_t)sample(A.c[2], x, y), m) << 16 | 0xFF000000u;
    } else {
        px = ycbcr_to_rgba(sample(A.c[0], x, y), sample(A.c[1], x, y), sample(A.c[2], x, y));
        if (A.color == TRT_JPEG_YCCK) {
            const uint32_t m = (uint32_t)sample(A.c[3], x, y);
            px = blinn(255u - (px & 255u), m) | blinn(255u - ((px >> 8) & 255u), m) << 8 |
                 blinn(255u - ((px >> 16) & 255u), m) << 16 | 0xFF000000u;
        }
    }
    A.out[(size_t)y * A.width + x] = px;
}

// The vertical source rows of stb's line-buffer walk (load_jpeg_image: ystep / ypos /
// line0 / line1): for every output row, the "near" and "far" sample rows.
std::vector<int32_t> walk_rows(int height, int vs, int px_h) {
    std::vector<int32_t> rows(2 * (size_t)height);
    int ystep = vs >> 1, line0 = 0, line1 = 0, ypos = 0;
    for (int j = 0; j < height; ++j) {
        const bool bottom = ystep >= (vs >> 1);
        rows[2 * j] = bottom ? line1 : line0;
        rows[2 * j + 1] = bottom ? line0 : line1;
        if (++ystep >= vs) {
            ystep = 0;
            line0 = line1;
            if (++ypos < px_h) ++line1;
        }
    }
    return rows;
}

template <class T>
hipError_t upload(T** d, const T* h, size_t n, hipStream_t s) {
    hipError_t e = hipMalloc(reinterpret_cast<void**>(d), n * sizeof(T));
    if (e != hipSuccess) return e;
    return hipMemcpyAsync(*d, h, n * sizeof(T), hipMemcpyHostToDevice, s);
}

} // namespace

hipError_t reconstruct(const Image& img, uint8_t* out_rgba8, hipStream_t stream) {
    const int nc = img.ncomp;
    int16_t* d_coef[4] = {};
    uint16_t* d_quant[4] = {};
    uint8_t* d_samples[4] = {};
    int32_t* d_rows[4] = {};
    hipError_t e = hipSuccess;
    ColorArgs A{};
    A.out = reinterpret_cast<uint32_t*>(out_rgba8);
    A.width = img.width;
    A.height = img.height;
    A.ncomp = nc;
    A.color = img.color;
    std::vector<int32_t> rows[4];
    for (int k = 0; k < nc && e == hipSuccess; ++k) {
        const Plane& p = img.comp[k];
        const uint32_t nblocks = (uint32_t)p.bw * (uint32_t)p.bh, stride = 8u * (uint32_t)p.bw;
        if ((e = upload(&d_coef[k], p.coef.data(), p.coef.size(), stream)) != hipSuccess) break;
        if ((e = upload(&d_quant[k], p.quant, 64, stream)) != hipSuccess) break;
        if ((e = hipMalloc(reinterpret_cast<void**>(&d_samples[k]), (size_t)nblocks * 64)) != hipSuccess) break;
        const uint32_t groups = (nblocks + kBlocksPerGroup - 1) / kBlocksPerGroup;
        hipLaunchKernelGGL(idct_kernel, dim3(groups), dim3(256), 0, stream, d_coef[k], d_quant[k], d_samples[k],
                           nblocks, (uint32_t)p.bw, stride);
        if ((e = hipGetLastError()) != hipSuccess) break;
        // the resampler of component k (load_jpeg_image: hs, vs are integer ratios)
        const int hs = img.hmax / p.h, vs = img.vmax / p.v;
        CompArgs& a = A.c[k];
        a.samples = d_samples[k];
        a.stride = stride;
        a.hs = hs;
        a.w_lores = (img.width + hs - 1) / hs;
        a.filter = (hs == 1 && vs == 1) ? F_COPY
                   : (hs == 1 && vs == 2) ? F_V2
                   : (hs == 2 && vs == 1) ? F_H2
                   : (hs == 2 && vs == 2) ? F_HV2
                                          : F_NEAREST;
        rows[k] = walk_rows(img.height, vs, p.px_h);
        if ((e = upload(&d_rows[k], rows[k].data(), rows[k].size(), stream)) != hipSuccess) break;
        a.rows = d_rows[k];
    }
    if (e == hipSuccess) {
        hipLaunchKernelGGL(color_kernel, dim3((img.width + 63) / 64, (img.height + 3) / 4), dim3(256), 0, stream, A);
        e = hipGetLastError();
    }
    const hipError_t s = hipStreamSynchronize(stream); // scratch is freed below
    if (e == hipSuccess) e = s;
    for (int k = 0; k < 4; ++k) {
        (void)hipFree(d_coef[k]);
        (void)hipFree(d_quant[k]);
        (void)hipFree(d_samples[k]);
        (void)hipFree(d_rows[k]);
    }
    return e;
}

} // namespace jpeg
} // namespace trt
