// bvh_build.cpp — binned-SAH BVH2 over the triangles of the uploaded batches.
//
// The reference tests every batch box and then every triangle of the batches it enters, in
// index order (shader.comp:338-361).  For incoherent secondary rays the wave-coherent batch
// walk pays for the union of the batches 64 lanes enter, so mesh scenes are traced per lane
// through this BVH instead.  The BVH is culling only — the kernel reproduces the reference's
// decision exactly:
//   * a triangle candidate counts only if ray_aabb_intersect of ITS batch box passes (the same
//     slab test the reference gates the triangle loop with);
//   * ties in t are broken by (batch, triangle) index, i.e. the first candidate in the
//     reference's loop order wins, as with its strict `t < nearest` update;
//   * node boxes are the triangles' exact bounds padded by max(1e-4 * extent, 1e-5 * |coord|,
//     1e-6) per axis, a margin far above MT / slab rounding, so neither a box miss nor the
//     distance pruning (skip a node entered beyond the best t) can drop a candidate the
//     reference would have taken.
// Built only when the batch ranges are disjoint (each triangle in at most one batch, true for
// every scene the reference's host code builds); otherwise the batch walk is used.
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <unordered_map>
#include <vector>

#include "../../include/trt/abi.h"
#include "trt_device.h"

namespace trt {

namespace {

struct Box {
    float lo[3], hi[3];
    void reset() {
        for (int k = 0; k < 3; ++k) {
            lo[k] = std::numeric_limits<float>::infinity();
            hi[k] = -std::numeric_limits<float>::infinity();
        }
    }
    void grow(const Box& b) {
        for (int k = 0; k < 3; ++k) {
            lo[k] = std::min(lo[k], b.lo[k]);
            hi[k] = std::max(hi[k], b.hi[k]);
        }
    }
    float area() const {
        float d[3];
        for (int k = 0; k < 3; ++k) d[k] = std::max(0.0f, hi[k] - lo[k]);
        return 2.0f * (d[0] * d[1] + d[1] * d[2] + d[2] * d[0]);
    }
};

struct Prim {
    Box box;
    float c[3]; // centroid
    uint32_t tri, batch, ni;
};

// SAH knobs: cost of one node visit in triangle tests (the split pays ct * parent area) and the
// leaf bounds.  Overridable for tuning (TRT_BVH_CT, TRT_BVH_LEAF_MIN, TRT_BVH_LEAF_MAX).
struct SahParams {
    float ct = 0.0f;
    uint32_t leaf_min = kBvhLeafMin, leaf_max = kBvhLeafMax;
    // Binned SAH over every axis with 32 bins (round 5; TRT_BVH_AXES=1 / TRT_BVH_BINS=16 give the
    // widest-centroid-axis, 16-bin build of rounds 1-4): C4 -0.8 %, C3 -1 %, the shipped frame and
    // the README scene -5 % (profiles/r05g_ab_codesize_bvh.jsonl)
    int all_axes = 1;
    int bins = 32;
    SahParams() {
        if (const char* e = std::getenv("TRT_BVH_AXES")) all_axes = std::atoi(e) == 3;
        if (const char* e = std::getenv("TRT_BVH_BINS")) bins = std::min(64, std::max(4, std::atoi(e)));
        if (const char* e = std::getenv("TRT_BVH_CT")) ct = std::strtof(e, nullptr);
        if (const char* e = std::getenv("TRT_BVH_LEAF_MIN")) leaf_min = (uint32_t)std::strtoul(e, nullptr, 10);
        if (const char* e = std::getenv("TRT_BVH_LEAF_MAX")) leaf_max = (uint32_t)std::strtoul(e, nullptr, 10);
        leaf_max = std::min<uint32_t>(std::max<uint32_t>(leaf_max, 1u), 16u); // 4-bit leaf count field
        leaf_min = std::min(std::max<uint32_t>(leaf_min, 1u), leaf_max);
    }
};

struct Builder {
    SahParams sp;
    std::vector<Prim> prims;
    std::vector<BvhNode> nodes;
    std::vector<uint32_t> order;

    // Returns the child reference (node index, or leaf encoding) for prims [b, e).
    uint32_t build(uint32_t b, uint32_t e, Box& out_box, int depth) {
        Box bb, cb;
        bb.reset();
        cb.reset();
        for (uint32_t i = b; i < e; ++i) {
            bb.grow(prims[i].box);
            Box c{{prims[i].c[0], prims[i].c[1], prims[i].c[2]}, {prims[i].c[0], prims[i].c[1], prims[i].c[2]}};
            cb.grow(c);
        }
        out_box = bb;
        const uint32_t n = e - b;
        if (n <= sp.leaf_min) return make_leaf(b, e);
        const bool median_only = depth >= kBvhSahDepth; // bounds the depth: <= 32 + log2(n) levels
        // binned SAH over the widest centroid axis (or every axis, all_axes)
        int axis = 0;
        float ext = cb.hi[0] - cb.lo[0];
        for (int k = 1; k < 3; ++k)
            if (cb.hi[k] - cb.lo[k] > ext) {
                ext = cb.hi[k] - cb.lo[k];
                axis = k;
            }
        uint32_t mid = b + n / 2;
        if (ext > 0.0f && !median_only) {
            constexpr int MAXB = 64;
            const int NB = sp.bins;
            float best = std::numeric_limits<float>::infinity();
            int best_k = -1, best_axis = axis;
            for (int a = 0; a < 3; ++a) {
                if (!sp.all_axes && a != axis) continue;
                const float ea = cb.hi[a] - cb.lo[a];
                if (!(ea > 0.0f)) continue;
                Box bins[MAXB];
                uint32_t cnt[MAXB] = {0};
                for (int k = 0; k < NB; ++k) bins[k].reset();
                const float scale = NB / ea;
                for (uint32_t i = b; i < e; ++i) {
                    int k = std::min(NB - 1, std::max(0, (int)((prims[i].c[a] - cb.lo[a]) * scale)));
                    bins[k].grow(prims[i].box);
                    cnt[k]++;
                }
                // right-hand sweeps once, then the left-to-right scan
                Box rsum[MAXB];
                uint32_t rcnt[MAXB];
                Box acc;
                acc.reset();
                uint32_t ac = 0;
                for (int k = NB - 1; k >= 0; --k) {
                    acc.grow(bins[k]);
                    ac += cnt[k];
                    rsum[k] = acc;
                    rcnt[k] = ac;
                }
                Box left;
                left.reset();
                uint32_t nl = 0;
                for (int k = 0; k < NB - 1; ++k) {
                    left.grow(bins[k]);
                    nl += cnt[k];
                    const uint32_t nr = rcnt[k + 1];
                    if (!nl || !nr) continue;
                    const float cost = sp.ct * bb.area() + left.area() * nl + rsum[k + 1].area() * nr;
                    if (cost < best) {
                        best = cost;
                        best_k = k;
                        best_axis = a;
                    }
                }
            }
            const float leaf_cost = bb.area() * n;
            if (n <= sp.leaf_max && !(best < leaf_cost)) return make_leaf(b, e);
            if (best_k >= 0) {
                const int a = best_axis;
                const float scale = NB / (cb.hi[a] - cb.lo[a]);
                auto it = std::partition(prims.begin() + b, prims.begin() + e, [&](const Prim& p) {
                    return std::min(NB - 1, std::max(0, (int)((p.c[a] - cb.lo[a]) * scale))) <= best_k;
                });
                mid = (uint32_t)(it - prims.begin());
                if (mid == b || mid == e) mid = b + n / 2;
                else axis = a;
            }
        }
        if (mid == b + n / 2) {
            std::nth_element(prims.begin() + b, prims.begin() + mid, prims.begin() + e,
                             [&](const Prim& x, const Prim& y) { return x.c[axis] < y.c[axis]; });
        }
        const uint32_t idx = (uint32_t)nodes.size();
        nodes.emplace_back();
        Box lb, rb;
        const uint32_t l = build(b, mid, lb, depth + 1);
        const uint32_t r = build(mid, e, rb, depth + 1);
        BvhNode& nd = nodes[idx];
        for (int k = 0; k < 3; ++k) {
            nd.lo0[k] = lb.lo[k];
            nd.hi0[k] = lb.hi[k];
            nd.lo1[k] = rb.lo[k];
            nd.hi1[k] = rb.hi[k];
        }
        nd.child[0] = l;
        nd.child[1] = r;
        return idx;
    }

    uint32_t make_leaf(uint32_t b, uint32_t e) { // 1 <= e - b <= sp.leaf_max <= 16
        const uint32_t start = (uint32_t)order.size();
        for (uint32_t i = b; i < e; ++i) order.push_back(i);
        return kBvhLeafBit | ((e - b - 1u) << kBvhCountShift) | start;
    }
};

// ---- spatial splits (Stich, Friedrich, Dietrich, "Spatial Splits in Bounding Volume
// Hierarchies", HPG 2009) ------------------------------------------------------------------
//
// A node may also split SPACE: a plane through the node's box, every triangle reference left or
// right of it, and a triangle crossing it referenced on both sides with its box clipped to each
// side.  Long thin triangles (the lathed glass of the shipped scene) otherwise give overlapping
// sibling boxes that incoherent rays inside the glass must all enter.  A reference is still the
// whole triangle (the kernel tests the triangle, not its clipped part), only the node boxes are
// tighter; a clipped box contains the triangle's part on its side of the plane (clipped in double,
// then padded like tri_box), so a ray hitting the triangle enters a box holding a reference to it.
// Duplicate references of one triangle return the same t and (batch, triangle), so the kernel's
// tie-break keeps one.
struct V3d {
    double x[3];
};

// Bounding box of the part of triangle t inside the slab lo <= x[a] <= hi (empty: lo > hi).
Box clip_box(const trt_triangle& t, int a, double lo, double hi) {
    V3d poly[9], tmp[9];
    int n = 3;
    const trt_vec4* v[3] = {&t.v0, &t.v1, &t.v2};
    for (int i = 0; i < 3; ++i)
        for (int k = 0; k < 3; ++k) poly[i].x[k] = (&v[i]->x)[k];
    auto clip = [&](double plane, bool keep_ge) {
        int m = 0;
        for (int i = 0; i < n; ++i) {
            const V3d& p = poly[i];
            const V3d& q = poly[(i + 1) % n];
            const bool pin = keep_ge ? p.x[a] >= plane : p.x[a] <= plane;
            const bool qin = keep_ge ? q.x[a] >= plane : q.x[a] <= plane;
            if (pin) tmp[m++] = p;
            if (pin != qin) {
                const double s = (plane - p.x[a]) / (q.x[a] - p.x[a]);
                V3d r;
                for (int k = 0; k < 3; ++k) r.x[k] = p.x[k] + s * (q.x[k] - p.x[k]);
                r.x[a] = plane;
                tmp[m++] = r;
            }
        }
        n = m;
        for (int i = 0; i < n; ++i) poly[i] = tmp[i];
    };
    clip(lo, true);
    if (n) clip(hi, false);
    Box b;
    b.reset();
    if (!n) return b;
    // outward rounding to float plus tri_box's padding of the whole triangle
    float tlo[3], thi[3];
    for (int k = 0; k < 3; ++k) {
        const float c0 = (&t.v0.x)[k], c1 = (&t.v1.x)[k], c2 = (&t.v2.x)[k];
        tlo[k] = std::min({c0, c1, c2});
        thi[k] = std::max({c0, c1, c2});
        double l = poly[0].x[k], h = poly[0].x[k];
        for (int i = 1; i < n; ++i) {
            l = std::min(l, poly[i].x[k]);
            h = std::max(h, poly[i].x[k]);
        }
        const float pad = std::max({1e-4f * (thi[k] - tlo[k]), 1e-5f * std::max(std::fabs(tlo[k]), std::fabs(thi[k])), 1e-6f});
        float lf = (float)l, hf = (float)h;
        if ((double)lf > l) lf = std::nextafter(lf, -std::numeric_limits<float>::infinity());
        if ((double)hf < h) hf = std::nextafter(hf, std::numeric_limits<float>::infinity());
        b.lo[k] = lf - pad;
        b.hi[k] = hf + pad;
    }
    return b;
}

Box intersect(const Box& a, const Box& b) {
    Box r;
    for (int k = 0; k < 3; ++k) {
        r.lo[k] = std::max(a.lo[k], b.lo[k]);
        r.hi[k] = std::min(a.hi[k], b.hi[k]);
    }
    return r;
}
bool empty_box(const Box& b) { return !(b.lo[0] <= b.hi[0] && b.lo[1] <= b.hi[1] && b.lo[2] <= b.hi[2]); }

struct SplitBuilder {
    SahParams sp;
    const trt_triangle* tris = nullptr;
    std::vector<BvhNode> nodes;
    std::vector<Prim> leaf_refs;
    float alpha = 1e-5f;     // spatial splits are tried when the object split's child overlap
    float root_area = 0.0f;  // exceeds alpha x the root's area (Stich et al.)
    size_t budget = 0;       // reference duplicates allowed in all (bounds the memory)

    uint32_t make_leaf(const std::vector<Prim>& refs) {
        const uint32_t start = (uint32_t)leaf_refs.size();
        leaf_refs.insert(leaf_refs.end(), refs.begin(), refs.end());
        return kBvhLeafBit | ((uint32_t)(refs.size() - 1u) << kBvhCountShift) | start;
    }

    uint32_t build(std::vector<Prim>& refs, Box& out_box, int depth) {
        Box bb, cb;
        bb.reset();
        cb.reset();
        for (const Prim& p : refs) {
            bb.grow(p.box);
            Box c{{p.c[0], p.c[1], p.c[2]}, {p.c[0], p.c[1], p.c[2]}};
            cb.grow(c);
        }
        out_box = bb;
        const uint32_t n = (uint32_t)refs.size();
        if (n <= sp.leaf_min) return make_leaf(refs);
        constexpr int NB = 32;
        // -- object split: binned SAH over every centroid axis --
        float best = std::numeric_limits<float>::infinity();
        int best_axis = -1, best_k = -1;
        Box best_l, best_r;
        for (int a = 0; a < 3 && depth < kBvhSahDepth; ++a) {
            const float ea = cb.hi[a] - cb.lo[a];
            if (!(ea > 0.0f)) continue;
            Box bins[NB];
            uint32_t cnt[NB] = {0};
            for (auto& x : bins) x.reset();
            const float scale = NB / ea;
            for (const Prim& p : refs) {
                const int k = std::min(NB - 1, std::max(0, (int)((p.c[a] - cb.lo[a]) * scale)));
                bins[k].grow(p.box);
                cnt[k]++;
            }
            Box rsum[NB];
            uint32_t rcnt[NB];
            Box acc;
            acc.reset();
            uint32_t ac = 0;
            for (int k = NB - 1; k >= 0; --k) {
                acc.grow(bins[k]);
                ac += cnt[k];
                rsum[k] = acc;
                rcnt[k] = ac;
            }
            Box left;
            left.reset();
            uint32_t nl = 0;
            for (int k = 0; k < NB - 1; ++k) {
                left.grow(bins[k]);
                nl += cnt[k];
                const uint32_t nr = rcnt[k + 1];
                if (!nl || !nr) continue;
                const float cost = left.area() * nl + rsum[k + 1].area() * nr;
                if (cost < best) {
                    best = cost;
                    best_axis = a;
                    best_k = k;
                    best_l = left;
                    best_r = rsum[k + 1];
                }
            }
        }
        // -- spatial split: chopped binning over every axis of the node box --
        float sbest = std::numeric_limits<float>::infinity();
        int s_axis = -1;
        double s_plane = 0.0;
        // Past kBvhSahDepth only median splits (as Builder): a binned split can peel off one bin
        // per level (geometrically spaced centroids), so without this the depth — and the BVH2
        // walk's stack, kBvhStack entries — would be unbounded.  With it: <= 32 + log2(n) + 1.
        if (depth >= kBvhSahDepth) best_axis = -1, best = std::numeric_limits<float>::infinity();
        bool try_spatial = depth < kBvhSahDepth && budget > 0;
        if (try_spatial && best_axis >= 0) {
            const Box ov = intersect(best_l, best_r);
            try_spatial = !empty_box(ov) && ov.area() > alpha * root_area;
        }
        if (try_spatial) {
            for (int a = 0; a < 3; ++a) {
                const double lo = bb.lo[a], ext = (double)bb.hi[a] - lo;
                if (!(ext > 0.0)) continue;
                Box bins[NB];
                uint32_t enter[NB] = {0}, exitc[NB] = {0};
                for (auto& x : bins) x.reset();
                auto bin_of = [&](double v) { return std::min(NB - 1, std::max(0, (int)((v - lo) / ext * NB))); };
                for (const Prim& p : refs) {
                    const int b0 = bin_of(p.box.lo[a]), b1 = bin_of(p.box.hi[a]);
                    enter[b0]++;
                    exitc[b1]++;
                    for (int k = b0; k <= b1; ++k) {
                        const double pl = lo + ext * k / NB, ph = lo + ext * (k + 1) / NB;
                        Box cbx = b0 == b1 ? p.box : intersect(clip_box(tris[p.tri], a, pl, ph), p.box);
                        if (!empty_box(cbx)) bins[k].grow(cbx);
                    }
                }
                Box rsum[NB];
                uint32_t rcnt[NB];
                Box acc;
                acc.reset();
                uint32_t ac = 0;
                for (int k = NB - 1; k >= 0; --k) {
                    acc.grow(bins[k]);
                    ac += exitc[k];
                    rsum[k] = acc;
                    rcnt[k] = ac;
                }
                Box left;
                left.reset();
                uint32_t nl = 0;
                for (int k = 0; k < NB - 1; ++k) {
                    left.grow(bins[k]);
                    nl += enter[k];
                    const uint32_t nr = rcnt[k + 1];
                    if (!nl || !nr) continue;
                    const float cost = left.area() * nl + rsum[k + 1].area() * nr;
                    if (cost < sbest) {
                        sbest = cost;
                        s_axis = a;
                        s_plane = lo + ext * (k + 1) / NB;
                    }
                }
            }
        }
        const float leaf_cost = bb.area() * n;
        const float split_cost = std::min(best, sbest);
        if (n <= sp.leaf_max && !(split_cost < leaf_cost)) return make_leaf(refs);
        std::vector<Prim> L, R;
        if (sbest < best && s_axis >= 0) {
            const int a = s_axis;
            for (const Prim& p : refs) {
                if ((double)p.box.hi[a] <= s_plane) {
                    L.push_back(p);
                } else if ((double)p.box.lo[a] >= s_plane) {
                    R.push_back(p);
                } else { // straddles: clipped to each side
                    Prim pl = p, pr = p;
                    pl.box = intersect(clip_box(tris[p.tri], a, -std::numeric_limits<double>::infinity(), s_plane), p.box);
                    pr.box = intersect(clip_box(tris[p.tri], a, s_plane, std::numeric_limits<double>::infinity()), p.box);
                    const bool el = empty_box(pl.box), er = empty_box(pr.box);
                    if (el && er) {
                        L.push_back(p);
                        continue;
                    }
                    for (Prim* q : {&pl, &pr})
                        for (int k = 0; k < 3; ++k) q->c[k] = 0.5f * (q->box.lo[k] + q->box.hi[k]);
                    if (!el) L.push_back(pl);
                    if (!er) R.push_back(pr);
                    if (!el && !er && budget) --budget;
                }
            }
            if (L.empty() || R.empty()) { // degenerate: fall back to the object split
                L.clear();
                R.clear();
                sbest = std::numeric_limits<float>::infinity();
            }
        }
        if (L.empty() && R.empty()) {
            if (best_axis >= 0) {
                const int a = best_axis;
                const float scale = NB / (cb.hi[a] - cb.lo[a]);
                for (const Prim& p : refs)
                    (std::min(NB - 1, std::max(0, (int)((p.c[a] - cb.lo[a]) * scale))) <= best_k ? L : R).push_back(p);
            }
            if (L.empty() || R.empty()) { // median on the widest centroid axis
                L.clear();
                R.clear();
                int a = 0;
                for (int k = 1; k < 3; ++k)
                    if (cb.hi[k] - cb.lo[k] > cb.hi[a] - cb.lo[a]) a = k;
                std::vector<Prim> v = refs;
                const size_t mid = v.size() / 2;
                std::nth_element(v.begin(), v.begin() + mid, v.end(),
                                 [&](const Prim& x, const Prim& y) { return x.c[a] < y.c[a]; });
                L.assign(v.begin(), v.begin() + mid);
                R.assign(v.begin() + mid, v.end());
            }
        }
        refs.clear();
        refs.shrink_to_fit();
        const uint32_t idx = (uint32_t)nodes.size();
        nodes.emplace_back();
        Box lb, rb;
        const uint32_t l = build(L, lb, depth + 1);
        const uint32_t r = build(R, rb, depth + 1);
        BvhNode& nd = nodes[idx];
        for (int k = 0; k < 3; ++k) {
            nd.lo0[k] = lb.lo[k];
            nd.hi0[k] = lb.hi[k];
            nd.lo1[k] = rb.lo[k];
            nd.hi1[k] = rb.hi[k];
        }
        nd.child[0] = l;
        nd.child[1] = r;
        return idx;
    }
};

Box tri_box(const trt_triangle& t) {
    Box b;
    const trt_vec4* v[3] = {&t.v0, &t.v1, &t.v2};
    for (int k = 0; k < 3; ++k) {
        float lo = std::numeric_limits<float>::infinity(), hi = -lo;
        for (int m = 0; m < 3; ++m) {
            const float c = (&v[m]->x)[k];
            lo = std::min(lo, c);
            hi = std::max(hi, c);
        }
        const float pad = std::max({1e-4f * (hi - lo), 1e-5f * std::max(std::fabs(lo), std::fabs(hi)), 1e-6f});
        b.lo[k] = lo - pad;
        b.hi[k] = hi + pad;
    }
    return b;
}

} // namespace

uint32_t bvh_depth(const std::vector<BvhNode>& b2);

// Returns false (no BVH) when batch ranges overlap, a triangle is NaN, or nothing is covered.
bool build_bvh(const trt_triangle* tris, uint32_t ntri, const trt_model* models, uint32_t nmodel,
               std::vector<BvhNode>& nodes, std::vector<TriGeo>& leaf_tris) {
    nodes.clear();
    leaf_tris.clear();
    std::vector<int32_t> owner(ntri, -1);
    for (uint32_t i = 0; i < nmodel; ++i) {
        const int32_t s = models[i].params0.x, n = models[i].params0.y;
        for (int32_t j = s; j < s + n; ++j) {
            if (owner[j] >= 0) return false; // overlapping batches: keep the batch walk
            owner[j] = (int32_t)i;
        }
    }
    // Spatial splits (SplitBuilder, up to 30 % more references; TRT_BVH_SPLITS=0 turns them off):
    // the shipped frame -7 %, the README scene -9.5 %, C3 / C4 unchanged (their uniform
    // icosphere triangles take no spatial split), profiles/r05g_ab_codesize_bvh.jsonl
    const char* sps = std::getenv("TRT_BVH_SPLITS");
    const bool spatial = !sps || std::atoi(sps) != 0;
    Builder B;
    for (uint32_t j = 0; j < ntri; ++j) {
        if (owner[j] < 0) continue; // never tested by the reference
        const trt_triangle& t = tris[j];
        for (const trt_vec4* v : {&t.v0, &t.v1, &t.v2})
            if (std::isnan(v->x) || std::isnan(v->y) || std::isnan(v->z)) return false;
        Prim p;
        p.box = tri_box(t);
        for (int k = 0; k < 3; ++k) p.c[k] = 0.5f * (p.box.lo[k] + p.box.hi[k]);
        p.tri = j;
        p.batch = (uint32_t)owner[j];
        p.ni = models[owner[j]].params0.z != 0 ? 1u : 0u;
        B.prims.push_back(p);
    }
    if (B.prims.empty()) return false;
    Box root;
    uint32_t r;
    std::vector<Prim> refs_out;
    if (spatial) {
        SplitBuilder S;
        S.tris = tris;
        Box all;
        all.reset();
        for (const Prim& p : B.prims) all.grow(p.box);
        S.root_area = all.area();
        S.budget = B.prims.size() * 3 / 10;
        std::vector<Prim> refs = B.prims;
        r = S.build(refs, root, 0);
        B.nodes.swap(S.nodes);
        refs_out.swap(S.leaf_refs);
    } else {
        B.nodes.reserve(2 * B.prims.size() / B.sp.leaf_min + 2);
        r = B.build(0, (uint32_t)B.prims.size(), root, 0);
        refs_out.reserve(B.order.size());
        for (uint32_t k : B.order) refs_out.push_back(B.prims[k]);
    }
    if (r & kBvhLeafBit) { // single leaf: wrap it in a node with an empty second child
        BvhNode nd;
        for (int k = 0; k < 3; ++k) {
            nd.lo0[k] = root.lo[k];
            nd.hi0[k] = root.hi[k];
            // NaN on every axis: every slab product is NaN, so tnear <= tfar fails for any ray
            // (an inverted lo > hi box is not empty under NaN-ignoring min/max: it would act
            // like the box between the two planes and test the leaf twice)
            nd.lo1[k] = kBvh4EmptyCoord;
            nd.hi1[k] = kBvh4EmptyCoord;
        }
        nd.child[0] = r;
        nd.child[1] = kBvh4None; // collapse_bvh4 keeps it an unused slot
        B.nodes.insert(B.nodes.begin(), nd);
    }
    nodes.swap(B.nodes);
    if (bvh_depth(nodes) > (uint32_t)kBvhStack) { // cannot happen with the median tail; kept exact anyway
        nodes.clear();
        return false; // the batch walk (exact, no stack bound) traces the meshes
    }
    leaf_tris.resize(refs_out.size());
    for (size_t k = 0; k < refs_out.size(); ++k) {
        const Prim& p = refs_out[k];
        const trt_triangle& t = tris[p.tri];
        TriGeo& g = leaf_tris[k];
        g.v0[0] = t.v0.x;
        g.v0[1] = t.v0.y;
        g.v0[2] = t.v0.z;
        g.e1[0] = t.v1.x - t.v0.x; // the shader's own subtraction (shader.comp:230-231)
        g.e1[1] = t.v1.y - t.v0.y;
        g.e1[2] = t.v1.z - t.v0.z;
        g.e2[0] = t.v2.x - t.v0.x;
        g.e2[1] = t.v2.y - t.v0.y;
        g.e2[2] = t.v2.z - t.v0.z;
        uint32_t meta[3] = {p.tri, p.batch, p.ni};
        std::memcpy(g.pad, meta, sizeof(meta));
    }
    return true;
}

// Collapses the BVH2 into 4-wide nodes: a BVH4 node's children are the BVH2 subtrees reached
// by repeatedly opening the inner child of largest surface area (up to 4).  Leaves keep their
// encoding (same leaf triangle array).  Node 0 is the root.  Returns the traversal stack the
// 4-wide walk can need: the largest sum over a root-to-leaf path of (children - 1), since a
// visit pushes at most all but one of its children.
uint32_t collapse_bvh4(const std::vector<BvhNode>& b2, std::vector<Bvh4Node>& b4) {
    b4.clear();
    if (b2.empty()) return 0;
    struct Ref {
        uint32_t ref;
        Box box;
    };
    auto area = [](const Box& b) { return b.area(); };
    // children of BVH2 node n as refs with boxes
    auto kids = [&](uint32_t n, Ref out[2]) {
        const BvhNode& nd = b2[n];
        for (int k = 0; k < 3; ++k) {
            out[0].box.lo[k] = nd.lo0[k];
            out[0].box.hi[k] = nd.hi0[k];
            out[1].box.lo[k] = nd.lo1[k];
            out[1].box.hi[k] = nd.hi1[k];
        }
        out[0].ref = nd.child[0];
        out[1].ref = nd.child[1];
    };
    // BFS over BVH2 inner nodes that become BVH4 nodes
    std::vector<uint32_t> todo{0u};
    b4.reserve(b2.size() / 2 + 1);
    std::vector<uint32_t> index_of(b2.size(), kBvh4None);
    index_of[0] = 0;
    b4.emplace_back();
    for (size_t qi = 0; qi < todo.size(); ++qi) {
        const uint32_t n2 = todo[qi];
        Ref set[4];
        int cnt = 2;
        kids(n2, set);
        for (;;) { // open the largest inner child while there is room
            int best = -1;
            float ba = -1.0f;
            for (int i = 0; i < cnt; ++i)
                if (!(set[i].ref & kBvhLeafBit) && area(set[i].box) > ba) {
                    ba = area(set[i].box);
                    best = i;
                }
            if (best < 0 || cnt == 4) break;
            Ref two[2];
            kids(set[best].ref, two);
            set[best] = two[0];
            set[cnt++] = two[1];
        }
        Bvh4Node nd;
        for (int i = 0; i < 4; ++i) {
            if (i < cnt) {
                nd.lox[i] = set[i].box.lo[0];
                nd.loy[i] = set[i].box.lo[1];
                nd.loz[i] = set[i].box.lo[2];
                nd.hix[i] = set[i].box.hi[0];
                nd.hiy[i] = set[i].box.hi[1];
                nd.hiz[i] = set[i].box.hi[2];
                uint32_t r = set[i].ref;
                if (!(r & kBvhLeafBit)) {
                    if (index_of[r] == kBvh4None) {
                        index_of[r] = (uint32_t)b4.size();
                        b4.emplace_back();
                        todo.push_back(r);
                    }
                    r = index_of[r];
                }
                nd.child[i] = r;
            } else {
                // an empty slot: a box that is NaN on every axis, which no query can enter
                // (trt_device.h kBvh4EmptyCoord), so the kernel tests all four slots without
                // checking the ref
                nd.lox[i] = nd.loy[i] = nd.loz[i] = kBvh4EmptyCoord;
                nd.hix[i] = nd.hiy[i] = nd.hiz[i] = kBvh4EmptyCoord;
                nd.child[i] = kBvh4None;
            }
            nd.pad[i] = 0;
        }
        b4[index_of[n2]] = nd;
    }
    // stack bound, children before parents reversed: nodes were appended in BFS order
    std::vector<uint32_t> need(b4.size(), 0);
    for (size_t i = b4.size(); i-- > 0;) {
        const Bvh4Node& nd = b4[i];
        uint32_t cnt = 0, deepest = 0;
        for (int k = 0; k < 4; ++k) {
            if (nd.child[k] == kBvh4None) continue;
            ++cnt;
            if (!(nd.child[k] & kBvhLeafBit)) deepest = std::max(deepest, need[nd.child[k]]);
        }
        need[i] = (cnt ? cnt - 1 : 0) + deepest;
    }
    return need.empty() ? 0 : need[0];
}

// Quantizes every BVH4 node's child boxes to 8-bit planes on a per-node grid (trt_device.h
// Bvh4QNode).  Per axis the step is the power of two s >= extent / 250 of the node box [L, H]
// and the origin p <= L - s (rounded down), so lower planes round down and upper planes round
// up with one extra step of margin each.  Every quantized box is checked (exactly, in double)
// to contain its padded child box; returns false (no quantized BVH) if one does not.
bool quantize_bvh4(const std::vector<Bvh4Node>& b4, std::vector<Bvh4QNode>& out) {
    out.assign(b4.size(), Bvh4QNode{});
    for (size_t n = 0; n < b4.size(); ++n) {
        const Bvh4Node& nd = b4[n];
        Bvh4QNode& q = out[n];
        const float* lo[3] = {nd.lox, nd.loy, nd.loz};
        const float* hi[3] = {nd.hix, nd.hiy, nd.hiz};
        q.exps = 0;
        for (int a = 0; a < 3; ++a) {
            double L = std::numeric_limits<double>::infinity(), H = -L;
            for (int i = 0; i < 4; ++i) {
                if (nd.child[i] == kBvh4None) continue;
                if (!std::isfinite(lo[a][i]) || !std::isfinite(hi[a][i])) return false;
                L = std::min(L, (double)lo[a][i]);
                H = std::max(H, (double)hi[a][i]);
            }
            if (!(L <= H)) return false; // no used slot
            const double ext = std::max(H - L, 1e-30);
            int e = (int)std::ceil(std::log2(ext / 250.0));
            while (std::ldexp(250.0, e) < ext) ++e; // guard log2 rounding
            if (e < -126 || e > 127) return false;
            const double sd = std::ldexp(1.0, e);
            const double pd = L - sd;
            float pf = (float)pd;
            if ((double)pf > pd) pf = std::nextafter(pf, -std::numeric_limits<float>::infinity());
            q.p[a] = pf;
            q.exps |= (uint32_t)(e + 127) << (8 * a);
            uint32_t wl = 0, wh = 0;
            for (int i = 0; i < 4; ++i) {
                uint32_t ql = 255, qh = 0; // unused slot: inverted box
                if (nd.child[i] != kBvh4None) {
                    const double fl = std::floor(((double)lo[a][i] - (double)pf) / sd) - 1.0;
                    const double ch = std::ceil(((double)hi[a][i] - (double)pf) / sd) + 1.0;
                    ql = (uint32_t)std::min(255.0, std::max(0.0, fl));
                    qh = (uint32_t)std::min(255.0, std::max(0.0, ch));
                    // exact containment check of the decoded planes
                    if ((double)pf + ql * sd > (double)lo[a][i] || (double)pf + qh * sd < (double)hi[a][i]) return false;
                }
                wl |= ql << (8 * i);
                wh |= qh << (8 * i);
            }
            q.qlo[a] = wl;
            q.qhi[a] = wh;
        }
        q.pad[0] = q.pad[1] = 0;
        for (int i = 0; i < 4; ++i) q.child[i] = nd.child[i];
    }
    return true;
}

// Levels of the deepest leaf of the BVH2 (root = 1): the BVH2 walk's stack holds at most
// depth - 1 entries, so build_bvh keeps depth <= kBvhStack.
uint32_t bvh_depth(const std::vector<BvhNode>& b2) {
    if (b2.empty()) return 0;
    uint32_t best = 0;
    std::vector<std::pair<uint32_t, uint32_t>> st{{0u, 1u}};
    while (!st.empty()) {
        const auto [n, d] = st.back();
        st.pop_back();
        best = std::max(best, d);
        for (uint32_t c : b2[n].child)
            if (c != kBvh4None && !(c & kBvhLeafBit)) st.push_back({c, d + 1});
    }
    return best;
}

} // namespace trt
