// jpeg.h — private interface between the host entropy decoder (jpeg_entropy.cpp) and the GPU
// reconstruction kernels (jpeg_kernel.hip) of the envmap JPEG path.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <string>
#include <vector>

namespace trt {
namespace jpeg {

// One component after entropy decoding.
struct Plane {
    int h = 1, v = 1;       // sampling factors
    int px_w = 0, px_h = 0; // samples the image covers: ceil(W * h / hmax) x ceil(H * v / vmax)
    int bw = 0, bh = 0;     // MCU-padded block grid (blocks per row / column)
    uint16_t quant[64] = {};   // quantisation table, natural order
    std::vector<int16_t> coef; // bw * bh blocks x 64 raw coefficients, natural order
};

struct Image {
    int width = 0, height = 0, ncomp = 0, hmax = 1, vmax = 1;
    bool progressive = false;
    int color = 0; // TRT_JPEG_* colour model of the RGBA output
    Plane comp[4];
};

// Host: markers + Huffman / progressive entropy decode.  false + err on failure.
bool decode_entropy(const uint8_t* data, size_t len, Image& out, std::string& err);

// Device: dequantise + IDCT + upsample + colour convert into out_rgba8 (device pointer,
// width * height * 4 bytes).  Allocates and frees its own scratch; enqueues on `stream`
// and waits for it before freeing.
hipError_t reconstruct(const Image& img, uint8_t* out_rgba8, hipStream_t stream);

} // namespace jpeg
} // namespace trt
