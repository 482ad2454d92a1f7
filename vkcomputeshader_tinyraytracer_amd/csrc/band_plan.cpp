// band_plan.cpp — the exchange plan of a tiled frame batch (include/trt/abi.h trt_band_plan).
//
// The reference renders every frame on one GPU and presents it (main.cpp:2108-2131,
// 2181-2205).  The tiled path deals a frame's rows to band groups over the ranks
// (trt_bands.h); this file says, for a batch of frames, which compact band buffers travel from
// which rank to which frame's root and where they land.  trt_multi.cpp executes the plan over
// RCCL; a host with its own transport (the torch.distributed mirror, dist.py) executes the
// same list, so both move exactly the same bytes.  Pure host arithmetic: no HIP call.
#include <algorithm>
#include <vector>

#include "../../include/trt/abi.h"
#include "band_plan.h"
#include "trt_bands.h"

namespace trt {

int build_band_plan(uint32_t W, uint32_t H, uint32_t B, uint32_t N, uint32_t G, uint32_t first, uint32_t F,
                    int root, uint32_t flags, trt_band_layout& L, std::vector<trt_band_xfer>* xfers) {
    if (W == 0 || H == 0 || B == 0 || N == 0 || G == 0 || F == 0) return TRT_ERR_INVALID;
    if (root != TRT_ROOT_ROTATE && (root < 0 || (uint32_t)root >= N)) return TRT_ERR_INVALID;
    const uint32_t NG = N * G;
    L.groups = NG;
    L.max_rows = 0;
    for (uint32_t g = 0; g < NG; ++g) L.max_rows = std::max(L.max_rows, band_group_rows(H, B, NG, g));
    L.block_bytes = (uint64_t)L.max_rows * W * 4;
    L.local_bytes = (uint64_t)F * G * L.block_bytes;
    std::vector<uint32_t> rooted(N, 0);
    for (uint32_t f = 0; f < F; ++f) ++rooted[trt_frame_root(first + f, N, root)];
    L.gather_bytes = (uint64_t)*std::max_element(rooted.begin(), rooted.end()) * NG * L.block_bytes;
    if (!xfers) return TRT_OK;
    xfers->clear();
    // one transfer per (sender, root): every batch frame the root owns, all of the sender's
    // groups, contiguous on both ends (per-transfer overhead, not bytes, dominated the
    // per-frame, per-group exchange: profiles/r03_exchange_probe_per_group_transfers.log)
    const bool self = (flags & TRT_PLAN_SELF_GATHER) != 0;
    uint32_t off = 0;
    for (uint32_t r = 0; r < N; ++r) {
        const uint32_t J = rooted[r];
        if (J)
            for (uint32_t q = 0; q < N; ++q) {
                if (q == r && !self) continue;
                trt_band_xfer x{};
                x.src = q;
                x.dst = r;
                x.frames = J;
                x.groups = G;
                x.first_slot = off;
                x.src_offset = (uint64_t)off * G * L.block_bytes;
                x.dst_offset = (uint64_t)q * J * G * L.block_bytes;
                x.bytes = (uint64_t)J * G * L.block_bytes;
                xfers->push_back(x);
            }
        off += J;
    }
    return TRT_OK;
}

// Frame slots of a batch: frames ordered by root, so slot[f] = off_root(f) + (the frame's index
// among its root's frames); j[f] = that index.
void band_plan_slots(uint32_t N, uint32_t first, uint32_t F, int root, std::vector<uint32_t>& slot,
                     std::vector<uint32_t>& j) {
    std::vector<uint32_t> rooted(N, 0), off(N, 0);
    slot.assign(F, 0);
    j.assign(F, 0);
    for (uint32_t f = 0; f < F; ++f) j[f] = rooted[trt_frame_root(first + f, N, root)]++;
    for (uint32_t r = 1; r < N; ++r) off[r] = off[r - 1] + rooted[r - 1];
    for (uint32_t f = 0; f < F; ++f) slot[f] = off[trt_frame_root(first + f, N, root)] + j[f];
}

} // namespace trt

extern "C" {

uint32_t trt_frame_root(uint32_t frame, uint32_t nranks, int root) {
    if (root >= 0) return (uint32_t)root;
    return nranks ? frame % nranks : 0u;
}

uint32_t trt_band_frame_row(uint32_t k, uint32_t band_rows, uint32_t groups, uint32_t g) {
    if (band_rows == 0 || groups <= 1) return k;
    return trt::band_frame_row(k, band_rows, groups, g);
}

int trt_band_plan(uint32_t width, uint32_t height, uint32_t band_rows, uint32_t nranks, uint32_t groups_per_rank,
                  uint32_t first_frame, uint32_t nframes, int root, uint32_t flags, trt_band_layout* layout,
                  trt_band_xfer* xfers, uint32_t cap, uint32_t* count) {
    trt_band_layout L{};
    std::vector<trt_band_xfer> v;
    const int rc = trt::build_band_plan(width, height, band_rows, nranks, groups_per_rank, first_frame, nframes, root,
                                        flags, L, &v);
    if (rc != TRT_OK) return rc;
    if (layout) *layout = L;
    if (count) *count = (uint32_t)v.size();
    if (xfers)
        for (uint32_t i = 0; i < cap && i < v.size(); ++i) xfers[i] = v[i];
    return TRT_OK;
}

} // extern "C"
