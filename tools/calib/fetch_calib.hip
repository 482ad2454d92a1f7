// tools/calib/fetch_calib.hip — what FETCH_SIZE counts for the access patterns of this tracer
// (MI355X_MICROARCH.md: "On gfx950 FETCH_SIZE reports exactly 1/2 of the bytes of a wide coalesced
// streaming read ... Other access widths are uncalibrated: calibrate on a known byte count in your
// own access pattern").  One dispatch per pattern over a 4 GiB buffer (past the 256 MiB Infinity
// Cache, every line touched once per dispatch, a fresh region per dispatch):
//   0 stream   : 16 B per lane, consecutive (coalesced), 64 MiB
//   1 sparse128: 16 B per lane at a random distinct 128-B line, 1 Mi lines
//   2 pair128  : two lanes per random line, at byte 0 and 64 of it (both halves), 1 Mi lines
//   3 sparse64 : 16 B per lane at byte 0 of a random distinct line's first half only — as 1 but
//                the other lanes of the wave read byte 16 of the same line (64 B of it in 4 lanes)
//   4 gather16 : the envmap-like pattern: 16 B per lane, lanes of a wave spread over 8 lines
//                8 lanes per line at 16-B steps (128 B of each line read)
// Prints the bytes each dispatch requested; rocprofv3 gives FETCH_SIZE per dispatch.  Every
// dispatch also streams its offset array (8 B per lane, coalesced), counted at half its bytes,
// which the analysis subtracts.  Regions start on 4-KiB boundaries.  Result
// (profiles/r05j_fetch_calibration_aligned.log): patterns 1-4 are each one 64-B-counted request
// per 128-B line touched (sparse128, pair128 — both halves of a line — and sparse64 alike, and
// gather16 reading all 128 B), i.e. FETCH_SIZE = half of the lines' bytes for gathers as for
// streams.  (A first run with regions misaligned to 128 B, profiles/r05i_fetch_calibration.log,
// put the pair's halves on two lines and read as if each half were its own request.)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <numeric>
#include <algorithm>
#include <set>
#include <random>
#include <vector>

__global__ void gather(const uint4* __restrict__ buf, const uint64_t* __restrict__ off, uint32_t n, uint4* __restrict__ out) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint4 v = buf[off[i] / 16];
    if ((v.x ^ v.y ^ v.z ^ v.w) == 0x12345678u) out[i & 1023] = v; // keeps the load
}

int main() {
    const size_t bytes = 4ull << 30, lines = bytes / 128;
    uint4* buf;
    uint4* out;
    if (hipMalloc(&buf, bytes) != hipSuccess || hipMalloc(&out, 1024 * 16) != hipSuccess) return 1;
    hipMemset(buf, 1, bytes);
    std::mt19937_64 rng(7);
    const uint32_t N = 1u << 20;
    std::vector<uint64_t> perm(lines / 4); // a quarter of the lines per pattern region
    auto region = [&](int r) { return (uint64_t)r * (bytes / 5 / 4096 * 4096); };
    std::vector<std::vector<uint64_t>> offs(5);
    // 0 stream
    for (uint32_t i = 0; i < 4 * N; ++i) offs[0].push_back(region(0) + 16ull * i);
    // random distinct lines of a region
    auto rand_lines = [&](int r, uint32_t n) {
        std::vector<uint64_t> v(bytes / 5 / 128);
        std::iota(v.begin(), v.end(), 0);
        std::shuffle(v.begin(), v.end(), rng);
        v.resize(n);
        for (auto& x : v) x = region(r) + 128 * x;
        return v;
    };
    for (uint64_t l : rand_lines(1, N)) offs[1].push_back(l);
    for (uint64_t l : rand_lines(2, N)) { offs[2].push_back(l); offs[2].push_back(l + 64); }
    for (uint64_t l : rand_lines(3, N / 4))
        for (int k = 0; k < 4; ++k) offs[3].push_back(l + 16 * k);
    for (uint64_t l : rand_lines(4, N / 8))
        for (int k = 0; k < 8; ++k) offs[4].push_back(l + 16 * k);
    uint64_t* doff;
    size_t maxn = 0;
    for (auto& o : offs) maxn = std::max(maxn, o.size());
    if (hipMalloc(&doff, maxn * 8) != hipSuccess) return 1;
    const char* names[5] = {"stream", "sparse128", "pair128", "sparse64", "gather16"};
    for (int p = 0; p < 5; ++p) {
        hipMemcpy(doff, offs[p].data(), offs[p].size() * 8, hipMemcpyHostToDevice);
        hipDeviceSynchronize();
        const uint32_t n = (uint32_t)offs[p].size();
        hipLaunchKernelGGL(gather, dim3((n + 255) / 256), dim3(256), 0, 0, buf, doff, n, out);
        hipDeviceSynchronize();
        std::set<uint64_t>* dummy = nullptr;
        (void)dummy;
        // distinct 64-B and 128-B blocks the dispatch touched
        std::vector<uint64_t> b64, b128;
        for (uint64_t o : offs[p]) { b64.push_back(o / 64); b128.push_back(o / 128); }
        std::sort(b64.begin(), b64.end());
        std::sort(b128.begin(), b128.end());
        const size_t u64 = std::unique(b64.begin(), b64.end()) - b64.begin();
        const size_t u128 = std::unique(b128.begin(), b128.end()) - b128.begin();
        std::printf("{\"dispatch\": %d, \"pattern\": \"%s\", \"requested_bytes\": %llu, \"bytes_in_64B_blocks\": %llu, "
                    "\"bytes_in_128B_lines\": %llu}\n", p, names[p], (unsigned long long)n * 16ull,
                    (unsigned long long)u64 * 64ull, (unsigned long long)u128 * 128ull);
    }
    return 0;
}
