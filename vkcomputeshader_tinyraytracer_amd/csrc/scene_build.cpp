// scene_build.cpp — host scene build of the reference (the input side of the hot path).
//
// Mirrors, for one modelList entry (config.hpp:97-101), the body of the loop in
// createShaderStorageBuffers() (main.cpp:1533-1567):
//   loadObjAsTriangles  main.cpp:2290-2335 (obj_load.cpp)
//   transformTriangles  main.cpp:192-216   — glm's translate/rotate/scale and mat4*vec4
//   computeVertexNormals main.cpp:218-252  — per exact-position face-normal sums
//   64-triangle batches + per-batch AABB   main.cpp:1548-1566
// glm itself is not in this image: its arithmetic is restated below in the
// order glm 0.9.9 evaluates it (ext/matrix_transform.inl, detail/type_mat4x4.inl,
// detail/func_geometric.inl, detail/func_common.inl).
#include <cmath>
#include <cstring>
#include <new>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/trt/abi.h"

namespace trt {
int obj_load_triangles(const char* path, std::vector<float>& positions,
                       std::vector<uint32_t>& indices, std::string& err);
}

struct trt_scene {
    uint32_t batch_size = 64; // main.cpp:1549
    std::vector<trt_triangle> tris;
    std::vector<trt_model> models;
    std::string err;
};

namespace {

struct v4 {
    float x, y, z, w;
};
struct m4 {
    v4 c[4]; // glm is column-major: m[i] is column i
};

v4 v4add(v4 a, v4 b) { return {a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w}; }
v4 v4muls(v4 a, float s) { return {a.x * s, a.y * s, a.z * s, a.w * s}; }

m4 identity() {
    m4 m;
    m.c[0] = {1, 0, 0, 0};
    m.c[1] = {0, 1, 0, 0};
    m.c[2] = {0, 0, 1, 0};
    m.c[3] = {0, 0, 0, 1};
    return m;
}

// glm::translate: Result[3] = m[0] * v[0] + m[1] * v[1] + m[2] * v[2] + m[3]
m4 translate(const m4& m, const float v[3]) {
    m4 r = m;
    r.c[3] = v4add(v4add(v4add(v4muls(m.c[0], v[0]), v4muls(m.c[1], v[1])), v4muls(m.c[2], v[2])), m.c[3]);
    return r;
}

// glm::rotate(m, angle, axis) for a unit coordinate axis
m4 rotate(const m4& m, float angle, const float axis_in[3]) {
    const float a = angle;
    const float c = std::cos(a);
    const float s = std::sin(a);
    // axis = normalize(v): v * inversesqrt(dot(v, v))
    float d = (axis_in[0] * axis_in[0] + axis_in[1] * axis_in[1]) + axis_in[2] * axis_in[2];
    float inv = 1.0f / std::sqrt(d);
    float axis[3] = {axis_in[0] * inv, axis_in[1] * inv, axis_in[2] * inv};
    float temp[3] = {(1.0f - c) * axis[0], (1.0f - c) * axis[1], (1.0f - c) * axis[2]};
    float R[3][3];
    R[0][0] = c + temp[0] * axis[0];
    R[0][1] = temp[0] * axis[1] + s * axis[2];
    R[0][2] = temp[0] * axis[2] - s * axis[1];
    R[1][0] = temp[1] * axis[0] - s * axis[2];
    R[1][1] = c + temp[1] * axis[1];
    R[1][2] = temp[1] * axis[2] + s * axis[0];
    R[2][0] = temp[2] * axis[0] + s * axis[1];
    R[2][1] = temp[2] * axis[1] - s * axis[0];
    R[2][2] = c + temp[2] * axis[2];
    m4 r;
    for (int i = 0; i < 3; ++i)
        r.c[i] = v4add(v4add(v4muls(m.c[0], R[i][0]), v4muls(m.c[1], R[i][1])), v4muls(m.c[2], R[i][2]));
    r.c[3] = m.c[3];
    return r;
}

// glm::scale
m4 scale(const m4& m, const float v[3]) {
    m4 r;
    r.c[0] = v4muls(m.c[0], v[0]);
    r.c[1] = v4muls(m.c[1], v[1]);
    r.c[2] = v4muls(m.c[2], v[2]);
    r.c[3] = m.c[3];
    return r;
}

// mat4 * vec4 (type_mat4x4.inl): (m[0]*v.x + m[1]*v.y) + (m[2]*v.z + m[3]*v.w)
trt_vec4 mul(const m4& m, const trt_vec4& v) {
    v4 a0 = v4add(v4muls(m.c[0], v.x), v4muls(m.c[1], v.y));
    v4 a1 = v4add(v4muls(m.c[2], v.z), v4muls(m.c[3], v.w));
    v4 r = v4add(a0, a1);
    return {r.x, r.y, r.z, r.w};
}

float radians(float deg) { return deg * 0.01745329251994329576923690768489f; } // glm::radians

struct f3 {
    float x, y, z;
};
f3 cross(f3 a, f3 b) { return {a.y * b.z - b.y * a.z, a.z * b.x - b.z * a.x, a.x * b.y - b.x * a.y}; }
f3 normalize(f3 v) {
    float d = (v.x * v.x + v.y * v.y) + v.z * v.z;
    float inv = 1.0f / std::sqrt(d);
    return {v.x * inv, v.y * inv, v.z * inv};
}

// Key with vec4 == semantics (so +0 == -0); the hash folds -0 to +0 like std::hash<float>.
struct PosKey {
    float x, y, z, w;
    bool operator==(const PosKey& o) const { return x == o.x && y == o.y && z == o.z && w == o.w; }
};
struct PosHash {
    size_t operator()(const PosKey& k) const {
        auto h = [](float f) -> size_t {
            if (f == 0.0f) return 0;
            uint32_t u;
            std::memcpy(&u, &f, 4);
            return (size_t)u * 0x9E3779B97F4A7C15ull;
        };
        return h(k.x) ^ (h(k.y) << 1) ^ (h(k.z) << 2);
    }
};

// computeVertexNormals, main.cpp:218-252
void compute_vertex_normals(std::vector<trt_triangle>& tris) {
    std::unordered_map<PosKey, f3, PosHash> acc;
    acc.reserve(tris.size() * 2);
    auto key = [](const trt_vec4& v) { return PosKey{v.x, v.y, v.z, v.w}; };
    for (const trt_triangle& t : tris) {
        f3 e1 = {t.v1.x - t.v0.x, t.v1.y - t.v0.y, t.v1.z - t.v0.z};
        f3 e2 = {t.v2.x - t.v0.x, t.v2.y - t.v0.y, t.v2.z - t.v0.z};
        f3 fn = normalize(cross(e1, e2));
        for (const trt_vec4* v : {&t.v0, &t.v1, &t.v2}) {
            f3& a = acc[key(*v)]; // value-initialised to (0,0,0) like glm::vec3()
            a = {a.x + fn.x, a.y + fn.y, a.z + fn.z};
        }
    }
    for (trt_triangle& t : tris) {
        f3 n0 = normalize(acc[key(t.v0)]);
        f3 n1 = normalize(acc[key(t.v1)]);
        f3 n2 = normalize(acc[key(t.v2)]);
        t.v0_norm = {n0.x, n0.y, n0.z, 0.0f};
        t.v1_norm = {n1.x, n1.y, n1.z, 0.0f};
        t.v2_norm = {n2.x, n2.y, n2.z, 0.0f};
    }
}

// glm::min / glm::max (func_common.inl): min(x,y) = y < x ? y : x; max(x,y) = x < y ? y : x
float gmin(float x, float y) { return y < x ? y : x; }
float gmax(float x, float y) { return x < y ? y : x; }
trt_vec4 vmin(const trt_vec4& a, const trt_vec4& b) {
    return {gmin(a.x, b.x), gmin(a.y, b.y), gmin(a.z, b.z), gmin(a.w, b.w)};
}
trt_vec4 vmax(const trt_vec4& a, const trt_vec4& b) {
    return {gmax(a.x, b.x), gmax(a.y, b.y), gmax(a.z, b.z), gmax(a.w, b.w)};
}

int add_triangles(trt_scene* s, std::vector<trt_triangle>& mt, const trt_material& mat,
                  const float sc[3], const float rot[3], const float tr[3], int normal_interp) {
    // transformTriangles, main.cpp:192-216
    m4 M = identity();
    M = translate(M, tr);
    const float az[3] = {0, 0, 1}, ay[3] = {0, 1, 0}, ax[3] = {1, 0, 0};
    M = rotate(M, radians(rot[2]), az);
    M = rotate(M, radians(rot[1]), ay);
    M = rotate(M, radians(rot[0]), ax);
    M = scale(M, sc);
    for (trt_triangle& t : mt) {
        t.v0 = mul(M, t.v0);
        t.v1 = mul(M, t.v1);
        t.v2 = mul(M, t.v2);
    }
    if (normal_interp == 1) compute_vertex_normals(mt); // main.cpp:1541-1543
    // 64-triangle batches with their own AABB, main.cpp:1548-1566
    const size_t bs = s->batch_size;
    for (size_t i = 0; i < mt.size(); i += bs) {
        const size_t end = std::min(i + bs, mt.size());
        trt_model m;
        m.params0 = {0, 0, normal_interp, 0};
        const float fm = 3.402823466e+38f; // FLT_MAX, geometry.hpp:43-44
        m.bboxMin = {fm, fm, fm, fm};
        m.bboxMax = {-fm, -fm, -fm, -fm};
        m.material = mat;
        for (size_t j = i; j < end; ++j) {
            const trt_triangle& t = mt[j];
            m.bboxMin = vmin(m.bboxMin, vmin(t.v0, vmin(t.v1, t.v2)));
            m.bboxMax = vmax(m.bboxMax, vmax(t.v0, vmax(t.v1, t.v2)));
        }
        m.params0.x = (int32_t)s->tris.size();
        m.params0.y = (int32_t)(end - i);
        s->tris.insert(s->tris.end(), mt.begin() + (long)i, mt.begin() + (long)end);
        s->models.push_back(m);
    }
    return TRT_OK;
}

int make_triangles(trt_scene* s, const float* pos, uint32_t nverts, const uint32_t* idx,
                   uint32_t ntris, const trt_material& mat, std::vector<trt_triangle>& out) {
    out.resize(ntris);
    for (uint32_t f = 0; f < ntris; ++f) {
        trt_triangle& t = out[f];
        std::memset(&t, 0, sizeof(t));
        trt_vec4* vs[3] = {&t.v0, &t.v1, &t.v2};
        for (int k = 0; k < 3; ++k) {
            uint32_t vi = idx[3 * f + k];
            if (vi >= nverts) {
                s->err = "triangle " + std::to_string(f) + " references vertex " + std::to_string(vi) +
                         " of " + std::to_string(nverts);
                return TRT_ERR_INVALID;
            }
            *vs[k] = {pos[3 * vi], pos[3 * vi + 1], pos[3 * vi + 2], 1.0f};
        }
        t.material = mat; // loadObjAsTriangles: tri.material = mat, normals zero
    }
    return TRT_OK;
}

} // namespace

extern "C" {

int trt_scene_create(trt_scene** out) {
    if (!out) return TRT_ERR_INVALID;
    *out = new (std::nothrow) trt_scene();
    return *out ? TRT_OK : TRT_ERR_OOM;
}

void trt_scene_destroy(trt_scene* s) { delete s; }

const char* trt_scene_last_error(const trt_scene* s) { return s ? s->err.c_str() : "null scene"; }

int trt_scene_set_batch_size(trt_scene* s, uint32_t bs) {
    if (!s || bs == 0) return TRT_ERR_INVALID;
    s->batch_size = bs;
    return TRT_OK;
}

int trt_scene_add_mesh(trt_scene* s, const float* positions, uint32_t nverts, const uint32_t* indices,
                       uint32_t ntris, const trt_material* mat, const float sc[3], const float rot[3],
                       const float tr[3], int normal_interp) {
    if (!s) return TRT_ERR_INVALID;
    if (!mat || !sc || !rot || !tr || (ntris && (!indices || !positions))) {
        s->err = "trt_scene_add_mesh: null argument";
        return TRT_ERR_INVALID;
    }
    try {
        std::vector<trt_triangle> mt;
        int rc = make_triangles(s, positions, nverts, indices, ntris, *mat, mt);
        if (rc != TRT_OK) return rc;
        return add_triangles(s, mt, *mat, sc, rot, tr, normal_interp);
    } catch (const std::bad_alloc&) {
        s->err = "out of memory";
        return TRT_ERR_OOM;
    }
}

int trt_scene_add_obj(trt_scene* s, const char* path, const trt_material* mat, const float sc[3],
                      const float rot[3], const float tr[3], int normal_interp) {
    if (!s) return TRT_ERR_INVALID;
    if (!path || !mat || !sc || !rot || !tr) {
        s->err = "trt_scene_add_obj: null argument";
        return TRT_ERR_INVALID;
    }
    try {
        std::vector<float> pos;
        std::vector<uint32_t> idx;
        int rc = trt::obj_load_triangles(path, pos, idx, s->err);
        if (rc != TRT_OK) return rc;
        std::vector<trt_triangle> mt;
        rc = make_triangles(s, pos.data(), (uint32_t)(pos.size() / 3), idx.data(),
                            (uint32_t)(idx.size() / 3), *mat, mt);
        if (rc != TRT_OK) return rc;
        return add_triangles(s, mt, *mat, sc, rot, tr, normal_interp);
    } catch (const std::bad_alloc&) {
        s->err = "out of memory";
        return TRT_ERR_OOM;
    }
}

uint32_t trt_scene_triangle_count(const trt_scene* s) { return s ? (uint32_t)s->tris.size() : 0; }
uint32_t trt_scene_model_count(const trt_scene* s) { return s ? (uint32_t)s->models.size() : 0; }
const trt_triangle* trt_scene_triangles(const trt_scene* s) {
    return s && !s->tris.empty() ? s->tris.data() : nullptr;
}
const trt_model* trt_scene_models(const trt_scene* s) {
    return s && !s->models.empty() ? s->models.data() : nullptr;
}

} // extern "C"
