// jpeg_entropy.cpp — host half of the envmap JPEG decoder.
//
// The reference loads its envmap with stb_image v2.22 (stbi_load(..., STBI_rgb_alpha),
// main.cpp:928-949; the decoder is the vendored lib/stb_image.h, jpeg section).  Decoding is
// split the MI355X way:
//   * here, on the host: marker parsing and the serial Huffman / progressive-refinement
//     entropy decode into raw (not yet dequantised) coefficient planes, int16 per
//     coefficient, natural order, 64 per block, MCU-padded block grid per component;
//   * on the GPU (jpeg_kernel.hip): dequantisation, the 8x8 integer IDCT, chroma upsampling
//     and colour conversion, straight into the envmap's device buffer.
// The result is the exact RGBA8 image stbi_load returns: the coefficient values follow the
// JPEG standard's entropy decoding (baseline sequential and progressive, DC/AC first and
// refinement scans, EOB runs, restart intervals), and the arithmetic of the GPU half is the
// integer arithmetic of stb's kernels.  Where stb departs from the letter of the standard on
// damaged streams, this follows stb: bits past a marker read as zeros, a missing restart
// marker ends the scan, fill bytes (0xFF runs) are skipped.
//
// Supported as in stb: 8-bit baseline (SOF0/SOF1) and progressive (SOF2), 1, 3 or 4
// components, sampling factors 1..4.  Not supported (as in stb): arithmetic coding, 12-bit,
// lossless, hierarchical.
#include <algorithm>
#include <cstdint>
#include <cstring>
#include <new>
#include <string>
#include <vector>

#include "../../include/trt/abi.h"
#include "jpeg.h"

namespace trt {
namespace jpeg {

namespace {

constexpr int kFastBits = 9;

// zig-zag sequence position -> natural (row-major) index; entries past 63 clamp a corrupt
// run onto the last coefficient instead of writing outside the block
constexpr uint8_t kNatural[80] = {
    0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,  12, 19, 26, 33,
    40, 48, 41, 34, 27, 20, 13, 6,  7,  14, 21, 28, 35, 42, 49, 56, 57, 50, 43, 36,
    29, 22, 15, 23, 30, 37, 44, 51, 58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54,
    47, 55, 62, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63};

struct HuffTable {
    bool defined = false;
    uint8_t lut[1 << kFastBits]; // top kFastBits bits -> symbol index, 0xFF: longer code
    uint8_t len[256];            // code length of symbol index
    uint8_t sym[256];            // symbol value of symbol index
    uint32_t limit[18];          // (last code of each length + 1) << (16 - length)
    int32_t base[17];            // symbol index - code, per length
    int nsym = 0;

    bool build(const uint8_t counts[16], const uint8_t* values) {
        int k = 0;
        for (int l = 1; l <= 16; ++l)
            for (int i = 0; i < counts[l - 1]; ++i) {
                if (k >= 256) return false;
                len[k++] = (uint8_t)l;
            }
        nsym = k;
        std::memcpy(sym, values, (size_t)k);
        uint32_t code = 0;
        int idx = 0;
        std::memset(lut, 0xFF, sizeof lut);
        for (int l = 1; l <= 16; ++l) {
            base[l] = idx - (int32_t)code;
            while (idx < nsym && len[idx] == l) {
                if (l <= kFastBits) {
                    const uint32_t first = code << (kFastBits - l), span = 1u << (kFastBits - l);
                    for (uint32_t j = 0; j < span; ++j) lut[first + j] = (uint8_t)idx;
                }
                ++code;
                ++idx;
            }
            if (code > (1u << l)) return false; // over-subscribed lengths
            limit[l] = code << (16 - l);
            code <<= 1;
        }
        limit[17] = 0xFFFFFFFFu;
        defined = true;
        return true;
    }
};

struct Component {
    int id = 0, h = 1, v = 1, tq = 0;
    int dc_table = 0, ac_table = 0;
    int dc_pred = 0;
    int px_w = 0, px_h = 0; // samples covered by the image (ceil(W * h / hmax) ...)
    int bw = 0, bh = 0;     // MCU-padded block grid
    std::vector<int16_t> coef;
};

struct Error {
    std::string msg;
};

class Decoder {
  public:
    Decoder(const uint8_t* d, size_t n) : data_(d), size_(n) {}

    void run(Image& out) {
        if (marker() != 0xD8) fail("not a JPEG (no SOI marker)");
        int m = marker();
        while (!(m == 0xC0 || m == 0xC1 || m == 0xC2)) {
            if (m == 0xC3 || (m >= 0xC5 && m <= 0xCF && m != 0xC8 && m != 0xCC))
                fail("unsupported JPEG process (lossless / hierarchical / arithmetic coding)");
            segment(m);
            m = marker();
            while (m == kNoMarker) {
                if (pos_ >= size_) fail("no SOF marker");
                m = marker();
            }
        }
        progressive_ = (m == 0xC2);
        frame_header();
        m = marker();
        while (m != 0xD9) {
            if (m == 0xDA) {
                scan_header();
                entropy_scan();
                if (pending_ == kNoMarker) { // junk after the scan data: find the next marker
                    while (pos_ < size_) {
                        if (data_[pos_++] == 0xFF) {
                            pending_ = pos_ < size_ ? data_[pos_++] : kNoMarker;
                            break;
                        }
                    }
                }
            } else if (m == 0xDC) { // DNL
                if (get16() != 4 || get16() != (uint32_t)height_) fail("bad DNL segment");
            } else if (m == kNoMarker) {
                if (pos_ >= size_) fail("unexpected end of data (no EOI)");
            } else {
                segment(m);
            }
            m = marker();
        }
        export_image(out);
    }

  private:
    static constexpr int kNoMarker = 0xFF;

    const uint8_t* data_;
    size_t size_, pos_ = 0;
    HuffTable dc_[4], ac_[4];
    uint16_t quant_[4][64] = {};
    bool quant_defined_[4] = {};
    Component comp_[4];
    int ncomp_ = 0, width_ = 0, height_ = 0, hmax_ = 1, vmax_ = 1, mcux_ = 0, mcuy_ = 0;
    bool progressive_ = false;
    int restart_interval_ = 0;
    bool jfif_ = false;
    int app14_ = -1;
    int rgb_ids_ = 0;
    // scan state
    int scan_n_ = 0, order_[4] = {}, ss_ = 0, se_ = 63, ah_ = 0, al_ = 0;
    int eob_run_ = 0, todo_ = 0;
    // bit reader: `bits_` valid bits left-aligned in `acc_`
    uint32_t acc_ = 0;
    int bits_ = 0;
    int pending_ = kNoMarker; // marker met inside entropy-coded data
    bool stop_ = false;       // after a marker: feed zeros

    [[noreturn]] static void fail(const char* m) { throw Error{m}; }

    uint32_t get8() { return pos_ < size_ ? data_[pos_++] : 0u; }
    uint32_t get16() {
        uint32_t hi = get8();
        return (hi << 8) | get8();
    }
    void skip(size_t n) { pos_ = std::min(size_, pos_ + n); }

    // next marker code, or kNoMarker when the next byte is not 0xFF
    int marker() {
        if (pending_ != kNoMarker) {
            int m = pending_;
            pending_ = kNoMarker;
            return m;
        }
        if (get8() != 0xFF) return kNoMarker;
        uint32_t c;
        do c = get8();
        while (c == 0xFF && pos_ < size_);
        return (int)c;
    }

    void segment(int m) {
        switch (m) {
        case kNoMarker: fail("expected a marker");
        case 0xDD: // DRI
            if (get16() != 4) fail("bad DRI length");
            restart_interval_ = (int)get16();
            return;
        case 0xDB: { // DQT
            int left = (int)get16() - 2;
            while (left > 0) {
                const uint32_t pq = get8();
                const int prec = (int)(pq >> 4), t = (int)(pq & 15);
                if (prec > 1 || t > 3) fail("bad DQT table");
                for (int i = 0; i < 64; ++i) quant_[t][kNatural[i]] = (uint16_t)(prec ? get16() : get8());
                quant_defined_[t] = true;
                left -= prec ? 129 : 65;
            }
            if (left != 0) fail("bad DQT length");
            return;
        }
        case 0xC4: { // DHT
            int left = (int)get16() - 2;
            while (left > 0) {
                const uint32_t tc_th = get8();
                const int tc = (int)(tc_th >> 4), th = (int)(tc_th & 15);
                if (tc > 1 || th > 3) fail("bad DHT header");
                uint8_t counts[16], vals[256];
                int n = 0;
                for (int i = 0; i < 16; ++i) {
                    counts[i] = (uint8_t)get8();
                    n += counts[i];
                }
                if (n > 256) fail("bad DHT symbol count");
                for (int i = 0; i < n; ++i) vals[i] = (uint8_t)get8();
                if (!(tc ? ac_[th] : dc_[th]).build(counts, vals)) fail("bad Huffman code lengths");
                left -= 17 + n;
            }
            if (left != 0) fail("bad DHT length");
            return;
        }
        default: break;
        }
        if ((m >= 0xE0 && m <= 0xEF) || m == 0xFE) { // APPn / COM
            int len = (int)get16();
            if (len < 2) fail("bad APP/COM length");
            len -= 2;
            if (m == 0xE0 && len >= 5) {
                static const uint8_t tag[5] = {'J', 'F', 'I', 'F', 0};
                bool ok = true;
                for (int i = 0; i < 5; ++i) ok &= get8() == tag[i];
                len -= 5;
                if (ok) jfif_ = true;
            } else if (m == 0xEE && len >= 12) {
                static const uint8_t tag[6] = {'A', 'd', 'o', 'b', 'e', 0};
                bool ok = true;
                for (int i = 0; i < 6; ++i) ok &= get8() == tag[i];
                len -= 6;
                if (ok) {
                    get8();  // version
                    get16(); // flags0
                    get16(); // flags1
                    app14_ = (int)get8();
                    len -= 6;
                }
            }
            skip((size_t)len);
            return;
        }
        fail("unknown marker");
    }

    void frame_header() {
        const uint32_t len = get16();
        if (len < 11) fail("bad SOF length");
        if (get8() != 8) fail("only 8-bit JPEG is supported");
        height_ = (int)get16();
        width_ = (int)get16();
        if (height_ == 0) fail("JPEG with delayed height (DNL) is not supported");
        if (width_ == 0) fail("zero JPEG width");
        ncomp_ = (int)get8();
        if (ncomp_ != 1 && ncomp_ != 3 && ncomp_ != 4) fail("bad JPEG component count");
        if (len != 8u + 3u * (uint32_t)ncomp_) fail("bad SOF length");
        static const int rgb[3] = {'R', 'G', 'B'};
        for (int i = 0; i < ncomp_; ++i) {
            Component& c = comp_[i];
            c.id = (int)get8();
            if (ncomp_ == 3 && c.id == rgb[i]) ++rgb_ids_;
            const uint32_t hv = get8();
            c.h = (int)(hv >> 4);
            c.v = (int)(hv & 15);
            c.tq = (int)get8();
            if (c.h < 1 || c.h > 4 || c.v < 1 || c.v > 4) fail("bad sampling factor");
            if (c.tq > 3) fail("bad quantisation table id");
            hmax_ = std::max(hmax_, c.h);
            vmax_ = std::max(vmax_, c.v);
        }
        if ((uint64_t)width_ * (uint64_t)height_ > (1ull << 30)) fail("JPEG too large");
        mcux_ = (width_ + 8 * hmax_ - 1) / (8 * hmax_);
        mcuy_ = (height_ + 8 * vmax_ - 1) / (8 * vmax_);
        for (int i = 0; i < ncomp_; ++i) {
            Component& c = comp_[i];
            c.px_w = (width_ * c.h + hmax_ - 1) / hmax_;
            c.px_h = (height_ * c.v + vmax_ - 1) / vmax_;
            c.bw = mcux_ * c.h;
            c.bh = mcuy_ * c.v;
            c.coef.assign((size_t)c.bw * c.bh * 64, 0);
        }
    }

    void scan_header() {
        const uint32_t len = get16();
        scan_n_ = (int)get8();
        if (scan_n_ < 1 || scan_n_ > 4 || scan_n_ > ncomp_) fail("bad SOS component count");
        if (len != 6u + 2u * (uint32_t)scan_n_) fail("bad SOS length");
        for (int i = 0; i < scan_n_; ++i) {
            const int id = (int)get8();
            const uint32_t tables = get8();
            int which = 0;
            while (which < ncomp_ && comp_[which].id != id) ++which;
            if (which == ncomp_) fail("SOS names an unknown component");
            comp_[which].dc_table = (int)(tables >> 4);
            comp_[which].ac_table = (int)(tables & 15);
            if (comp_[which].dc_table > 3 || comp_[which].ac_table > 3) fail("bad Huffman table id");
            order_[i] = which;
        }
        ss_ = (int)get8();
        se_ = (int)get8();
        const uint32_t a = get8();
        ah_ = (int)(a >> 4);
        al_ = (int)(a & 15);
        if (progressive_) {
            if (ss_ > 63 || se_ > 63 || ss_ > se_ || ah_ > 13 || al_ > 13) fail("bad progressive SOS");
        } else {
            if (ss_ != 0 || ah_ != 0 || al_ != 0) fail("bad baseline SOS");
            se_ = 63;
        }
    }

    // ---- bits ------------------------------------------------------------------------------
    void refill() { // top up to >= 25 valid bits; after a marker, zeros
        while (bits_ <= 24) {
            uint32_t b = 0;
            if (!stop_) {
                b = get8();
                if (b == 0xFF) {
                    uint32_t c = get8();
                    while (c == 0xFF) c = get8();
                    if (c != 0) { // a marker: stop consuming, feed zeros
                        pending_ = (int)c;
                        stop_ = true;
                        return;
                    }
                }
            }
            acc_ |= b << (24 - bits_);
            bits_ += 8;
        }
    }
    uint32_t take(int n) { // n in 1..16
        if (bits_ < n) refill();
        const uint32_t v = acc_ >> (32 - n);
        acc_ <<= n;
        bits_ -= n;
        return v;
    }
    bool bit() { return take(1) != 0; }
    int receive_extend(int n) { // n in 1..15
        const uint32_t v = take(n);
        return (v >> (n - 1)) ? (int)v : (int)v - (1 << n) + 1;
    }
    int decode(const HuffTable& t) {
        if (!t.defined) fail("scan uses an undefined Huffman table");
        if (bits_ < 16) refill();
        const int k = t.lut[acc_ >> (32 - kFastBits)];
        if (k != 0xFF) {
            const int l = t.len[k];
            if (l > bits_) fail("bad Huffman code");
            acc_ <<= l;
            bits_ -= l;
            return t.sym[k];
        }
        const uint32_t top = acc_ >> 16;
        int l = kFastBits + 1;
        while (l <= 16 && top >= t.limit[l]) ++l;
        if (l > 16 || l > bits_) fail("bad Huffman code");
        const int idx = (int)(acc_ >> (32 - l)) + t.base[l];
        if (idx < 0 || idx >= t.nsym) fail("bad Huffman code");
        acc_ <<= l;
        bits_ -= l;
        return t.sym[idx];
    }

    void reset_interval() {
        acc_ = 0;
        bits_ = 0;
        stop_ = false;
        pending_ = kNoMarker;
        for (auto& c : comp_) c.dc_pred = 0;
        todo_ = restart_interval_ ? restart_interval_ : 0x7FFFFFFF;
        eob_run_ = 0;
    }

    // ---- blocks -------------------------------------------------------------------------
    void block_sequential(Component& c, int16_t* b) {
        const int t = decode(dc_[c.dc_table]);
        if (t > 15) fail("bad DC magnitude");
        c.dc_pred += t ? receive_extend(t) : 0;
        b[0] = (int16_t)c.dc_pred;
        const HuffTable& ac = ac_[c.ac_table];
        for (int k = 1; k < 64;) {
            const int rs = decode(ac);
            const int r = rs >> 4, s = rs & 15;
            if (s == 0) {
                if (rs != 0xF0) break; // EOB
                k += 16;
            } else {
                k += r;
                b[kNatural[k++]] = (int16_t)receive_extend(s);
            }
        }
    }

    void block_dc(Component& c, int16_t* b) {
        if (se_ != 0) fail("progressive scan mixes DC and AC");
        if (ah_ == 0) {
            const int t = decode(dc_[c.dc_table]);
            if (t > 15) fail("bad DC magnitude");
            c.dc_pred += t ? receive_extend(t) : 0;
            std::memset(b, 0, 64 * sizeof(int16_t));
            b[0] = (int16_t)(c.dc_pred * (1 << al_));
        } else if (bit()) {
            b[0] = (int16_t)(b[0] + (1 << al_));
        }
    }

    void refine(int16_t* p, int16_t step) {
        if (*p != 0 && bit() && (*p & step) == 0) *p = (int16_t)(*p > 0 ? *p + step : *p - step);
    }

    void block_ac(Component& c, int16_t* b) {
        if (ss_ == 0) fail("progressive scan mixes DC and AC");
        const HuffTable& ac = ac_[c.ac_table];
        if (ah_ == 0) { // first pass over this band
            if (eob_run_) {
                --eob_run_;
                return;
            }
            for (int k = ss_; k <= se_;) {
                const int rs = decode(ac);
                const int r = rs >> 4, s = rs & 15;
                if (s == 0) {
                    if (r < 15) {
                        eob_run_ = (1 << r) - 1 + (r ? (int)take(r) : 0);
                        break;
                    }
                    k += 16;
                } else {
                    k += r;
                    b[kNatural[k++]] = (int16_t)(receive_extend(s) * (1 << al_));
                }
            }
            return;
        }
        const int16_t step = (int16_t)(1 << al_); // refinement pass
        if (eob_run_) {
            --eob_run_;
            for (int k = ss_; k <= se_; ++k) refine(&b[kNatural[k]], step);
            return;
        }
        for (int k = ss_; k <= se_;) {
            const int rs = decode(ac);
            int r = rs >> 4;
            const int s = rs & 15;
            int16_t val = 0;
            if (s == 0) {
                if (r < 15) {
                    eob_run_ = (1 << r) - 1 + (r ? (int)take(r) : 0);
                    r = 64; // refine the rest of the band, then stop
                }
            } else {
                if (s != 1) fail("bad progressive refinement code");
                val = bit() ? step : (int16_t)-step;
            }
            while (k <= se_) {
                int16_t* p = &b[kNatural[k++]];
                if (*p != 0) {
                    refine(p, step);
                } else {
                    if (r == 0) {
                        *p = val;
                        break;
                    }
                    --r;
                }
            }
        }
    }

    void do_block(Component& c, int bx, int by) {
        int16_t* b = c.coef.data() + 64 * ((size_t)by * c.bw + bx);
        if (!progressive_) block_sequential(c, b);
        else if (ss_ == 0) block_dc(c, b);
        else block_ac(c, b);
    }

    // true: keep going; false: the interval ended without a restart marker (stb: stop)
    bool count_mcu() {
        if (--todo_ > 0) return true;
        if (bits_ < 24) refill();
        if (!(pending_ >= 0xD0 && pending_ <= 0xD7)) return false;
        reset_interval();
        return true;
    }

    void entropy_scan() {
        reset_interval();
        if (scan_n_ == 1) { // non-interleaved: the component's own block grid
            Component& c = comp_[order_[0]];
            const int w = (c.px_w + 7) >> 3, h = (c.px_h + 7) >> 3;
            for (int by = 0; by < h; ++by)
                for (int bx = 0; bx < w; ++bx) {
                    do_block(c, bx, by);
                    if (!count_mcu()) return;
                }
            return;
        }
        if (progressive_ && ss_ != 0) fail("interleaved progressive AC scan");
        for (int my = 0; my < mcuy_; ++my)
            for (int mx = 0; mx < mcux_; ++mx) {
                for (int k = 0; k < scan_n_; ++k) {
                    Component& c = comp_[order_[k]];
                    for (int y = 0; y < c.v; ++y)
                        for (int x = 0; x < c.h; ++x) do_block(c, mx * c.h + x, my * c.v + y);
                }
                if (!count_mcu()) return;
            }
    }

    void export_image(Image& out) {
        out.width = width_;
        out.height = height_;
        out.ncomp = ncomp_;
        out.progressive = progressive_;
        out.hmax = hmax_;
        out.vmax = vmax_;
        // colour model of stbi_load's STBI_rgb_alpha output (load_jpeg_image)
        if (ncomp_ == 1) out.color = TRT_JPEG_GRAY;
        else if (ncomp_ == 3) out.color = (rgb_ids_ == 3 || (app14_ == 0 && !jfif_)) ? TRT_JPEG_RGB : TRT_JPEG_YCBCR;
        else out.color = app14_ == 0 ? TRT_JPEG_CMYK : app14_ == 2 ? TRT_JPEG_YCCK : TRT_JPEG_YCBCR;
        for (int i = 0; i < ncomp_; ++i) {
            const Component& c = comp_[i];
            if (!quant_defined_[c.tq]) fail("component uses an undefined quantisation table");
            Plane& p = out.comp[i];
            p.h = c.h;
            p.v = c.v;
            p.px_w = c.px_w;
            p.px_h = c.px_h;
            p.bw = c.bw;
            p.bh = c.bh;
            std::memcpy(p.quant, quant_[c.tq], sizeof p.quant);
            p.coef = std::move(comp_[i].coef);
        }
    }
};

} // namespace

bool decode_entropy(const uint8_t* data, size_t len, Image& out, std::string& err) {
    try {
        Decoder d(data, len);
        d.run(out);
        return true;
    } catch (const Error& e) {
        err = e.msg;
    } catch (const std::bad_alloc&) {
        err = "out of memory";
    }
    return false;
}

} // namespace jpeg
} // namespace trt
