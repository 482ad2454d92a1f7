// jpeg_api.cpp — trt_jpeg_* handle functions of the C-ABI (host side of SURVEY §8 f2).
#include <cstring>
#include <new>
#include <string>

#include "../../include/trt/abi.h"
#include "jpeg.h"

struct trt_jpeg {
    trt::jpeg::Image img;
    bool parsed = false;
    std::string err;
};

namespace trt {
namespace jpeg {
const Image* image_of(const trt_jpeg* j) { return j && j->parsed ? &j->img : nullptr; }
} // namespace jpeg
} // namespace trt

extern "C" {

int trt_jpeg_create(trt_jpeg** out) {
    if (!out) return TRT_ERR_INVALID;
    *out = new (std::nothrow) trt_jpeg();
    return *out ? TRT_OK : TRT_ERR_OOM;
}

void trt_jpeg_destroy(trt_jpeg* j) { delete j; }

const char* trt_jpeg_last_error(const trt_jpeg* j) { return j ? j->err.c_str() : "null trt_jpeg"; }

int trt_jpeg_parse(trt_jpeg* j, const uint8_t* data, size_t len) {
    if (!j) return TRT_ERR_INVALID;
    j->parsed = false;
    j->img = trt::jpeg::Image();
    if (!data || len < 4) {
        j->err = "trt_jpeg_parse: no data";
        return TRT_ERR_INVALID;
    }
    if (!trt::jpeg::decode_entropy(data, len, j->img, j->err)) return TRT_ERR_IO;
    j->parsed = true;
    j->err.clear();
    return TRT_OK;
}

int trt_jpeg_get_info(const trt_jpeg* j, trt_jpeg_info* info) {
    if (!j || !info || !j->parsed) return TRT_ERR_INVALID;
    std::memset(info, 0, sizeof *info);
    const auto& im = j->img;
    info->width = (uint32_t)im.width;
    info->height = (uint32_t)im.height;
    info->components = (uint32_t)im.ncomp;
    info->progressive = im.progressive ? 1u : 0u;
    info->color = im.color;
    info->hmax = (uint32_t)im.hmax;
    info->vmax = (uint32_t)im.vmax;
    for (int k = 0; k < im.ncomp; ++k) {
        info->h[k] = (uint32_t)im.comp[k].h;
        info->v[k] = (uint32_t)im.comp[k].v;
        info->blocks_w[k] = (uint32_t)im.comp[k].bw;
        info->blocks_h[k] = (uint32_t)im.comp[k].bh;
    }
    return TRT_OK;
}

const int16_t* trt_jpeg_coefficients(const trt_jpeg* j, uint32_t c) {
    if (!j || !j->parsed || c >= (uint32_t)j->img.ncomp) return nullptr;
    return j->img.comp[c].coef.data();
}

const uint16_t* trt_jpeg_quant(const trt_jpeg* j, uint32_t c) {
    if (!j || !j->parsed || c >= (uint32_t)j->img.ncomp) return nullptr;
    return j->img.comp[c].quant;
}

} // extern "C"
