// tools/bvh_stats.cpp — offline quality of the product's BVH build (csrc/bvh_build.cpp) for a
// dumped scene: node / leaf counts and the SAH cost of the BVH4 the kernel walks (expected node
// visits and triangle tests of a random ray through the root box: sum over nodes of
// area / root area, and over leaves of area / root area x triangles).  Build knobs come from
// the environment as in the library.
//   tools/bvh_stats <tris.bin> <models.bin>   (trt_triangle / trt_model arrays, raw)
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../include/trt/abi.h"
#include "../include/trt/scene_types.h"
#include "../vkcomputeshader_tinyraytracer_amd/csrc/trt_device.h"

namespace trt {
bool build_bvh(const trt_triangle* tris, uint32_t ntri, const trt_model* models, uint32_t nmodel,
               std::vector<BvhNode>& nodes, std::vector<TriGeo>& leaf_tris);
uint32_t collapse_bvh4(const std::vector<BvhNode>& b2, std::vector<Bvh4Node>& b4);
}

template <class T>
static std::vector<T> load(const char* path) {
    std::vector<T> v;
    FILE* f = std::fopen(path, "rb");
    if (!f) { std::perror(path); std::exit(1); }
    std::fseek(f, 0, SEEK_END);
    const long n = std::ftell(f);
    std::fseek(f, 0, SEEK_SET);
    v.resize(n / sizeof(T));
    if (std::fread(v.data(), sizeof(T), v.size(), f) != v.size()) std::exit(1);
    std::fclose(f);
    return v;
}

static double area(float lx, float ly, float lz, float hx, float hy, float hz) {
    const double dx = hx - lx, dy = hy - ly, dz = hz - lz;
    return 2.0 * (dx * dy + dy * dz + dz * dx);
}

int main(int argc, char** argv) {
    if (argc < 3) return 2;
    auto tris = load<trt_triangle>(argv[1]);
    auto models = load<trt_model>(argv[2]);
    std::vector<trt::BvhNode> b2;
    std::vector<trt::TriGeo> lt;
    if (!trt::build_bvh(tris.data(), (uint32_t)tris.size(), models.data(), (uint32_t)models.size(), b2, lt)) return 3;
    std::vector<trt::Bvh4Node> b4;
    const uint32_t stack = trt::collapse_bvh4(b2, b4);
    // root box = union of the root's children
    const trt::Bvh4Node& r = b4[0];
    float L[3] = {1e30f, 1e30f, 1e30f}, H[3] = {-1e30f, -1e30f, -1e30f};
    for (int i = 0; i < 4; ++i) {
        if (r.child[i] == trt::kBvh4None) continue;
        L[0] = std::min(L[0], r.lox[i]); L[1] = std::min(L[1], r.loy[i]); L[2] = std::min(L[2], r.loz[i]);
        H[0] = std::max(H[0], r.hix[i]); H[1] = std::max(H[1], r.hiy[i]); H[2] = std::max(H[2], r.hiz[i]);
    }
    const double ra = area(L[0], L[1], L[2], H[0], H[1], H[2]);
    double visits = 1.0, tests = 0.0;
    size_t leaves = 0, leaf_tris = 0;
    for (const auto& n : b4)
        for (int i = 0; i < 4; ++i) {
            const uint32_t c = n.child[i];
            if (c == trt::kBvh4None) continue;
            const double a = area(n.lox[i], n.loy[i], n.loz[i], n.hix[i], n.hiy[i], n.hiz[i]) / ra;
            if (c & trt::kBvhLeafBit) {
                const uint32_t cnt = ((c >> trt::kBvhCountShift) & 15u) + 1u;
                tests += a * cnt;
                ++leaves;
                leaf_tris += cnt;
            } else {
                visits += a;
            }
        }
    std::printf("{\"tris\": %zu, \"bvh4_nodes\": %zu, \"leaves\": %zu, \"leaf_refs\": %zu, \"stack\": %u, "
                "\"sah_visits\": %.3f, \"sah_tri_tests\": %.3f}\n",
                tris.size(), b4.size(), leaves, leaf_tris, stack, visits, tests);
    return 0;
}
