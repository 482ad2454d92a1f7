// band_plan.h — internal entry to the exchange plan of a tiled batch (band_plan.cpp).
#pragma once

#include <vector>

#include "../../include/trt/abi.h"

namespace trt {

// The plan of include/trt/abi.h trt_band_plan into a vector (xfers may be null: layout only).
int build_band_plan(uint32_t W, uint32_t H, uint32_t B, uint32_t N, uint32_t G, uint32_t first, uint32_t F,
                    int root, uint32_t flags, trt_band_layout& L, std::vector<trt_band_xfer>* xfers);
// Frame slots of the plan's buffers: slot[f] (the sender's buffer) and j[f] (the frame's index
// among its root's frames of the batch).
void band_plan_slots(uint32_t N, uint32_t first, uint32_t F, int root, std::vector<uint32_t>& slot,
                     std::vector<uint32_t>& j);

} // namespace trt
