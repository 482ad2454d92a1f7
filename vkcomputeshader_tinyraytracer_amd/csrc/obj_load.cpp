// obj_load.cpp — OBJ -> triangle list with the semantics the reference relies on.
//
// The reference loads meshes with its vendored tinyobjloader (VCSA/lib/tiny_obj_loader.h,
// v2.0.x) via loadObjAsTriangles (main.cpp:2290-2335), which keeps only triangle faces in
// file order — and since LoadObj triangulates by default (tiny_obj_loader.h:611), every face
// arrives as triangles.  What decides the triangles is therefore tinyobj's behaviour, which
// is restated here (not linked; the library is not part of this build):
//   * `v x y z` numbers: its own decimal parser (tryParseDouble, :897-1028): integer and
//     fraction digits accumulated in double (fraction digit k weighted by 10^-k), decimal
//     exponent applied as ldexp(m * 5^e, e), then narrowed to float (parseReal, :1030-1038);
//   * `f` corners: atoi of each `v[/vt[/vn]]` triple, 1-based or negative-relative
//     (fixIndex, :819-850); a zero vertex index fails the load;
//   * quads: split on the shorter diagonal, ties -> [0,1,3],[1,2,3] (:1509-1616);
//   * n-gons: tinyobj's built-in ear clipper on the two dominant axes (:1740-1963) — the
//     mapbox earcut path is not compiled in the reference (TINYOBJLOADER_USE_MAPBOX_EARCUT
//     undefined).
// Checked bit-for-bit against the vendored library on every reference asset by
// tests/test_scene_build.py (goldens made by oracle/_ref/tinyobj_dump).
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <limits>
#include <string>
#include <vector>

#include "../../include/trt/abi.h"

namespace trt {

namespace {

inline bool is_digit(char c) { return (unsigned)(c - '0') < 10u; }
inline bool is_space(char c) { return c == ' ' || c == '\t'; }
inline bool is_eol(char c) { return c == '\r' || c == '\n' || c == '\0'; }

// tinyobj's tryParseDouble: greedy, stops at the first non-conforming character.
bool parse_double(const char* s, const char* end, double* out) {
    if (s >= end) return false;
    const char* p = s;
    double m = 0.0;
    int e10 = 0;
    char sign = '+';
    bool lead_dot = false;
    if (*p == '+' || *p == '-') {
        sign = *p++;
        if (p != end && *p == '.') lead_dot = true;
    } else if (*p == '.') {
        lead_dot = true;
    } else if (!is_digit(*p)) {
        return false;
    }
    bool more = p != end;
    if (!lead_dot) {
        int n = 0;
        while (more && is_digit(*p)) {
            m *= 10;
            m += (int)(*p - '0');
            ++p;
            ++n;
            more = p != end;
        }
        if (n == 0) return false;
    }
    if (more) {
        bool go_exp = false;
        if (*p == '.') {
            ++p;
            int k = 1;
            more = p != end;
            static const double lut[] = {1.0, 0.1, 0.01, 0.001, 0.0001, 0.00001, 0.000001, 0.0000001};
            while (more && is_digit(*p)) {
                m += (int)(*p - '0') * (k < 8 ? lut[k] : std::pow(10.0, -k));
                ++k;
                ++p;
                more = p != end;
            }
            go_exp = more;
        } else if (*p == 'e' || *p == 'E') {
            go_exp = true;
        }
        if (go_exp && (*p == 'e' || *p == 'E')) {
            ++p;
            more = p != end;
            char esign = '+';
            if (more && (*p == '+' || *p == '-')) {
                esign = *p++;
            } else if (!is_digit(*p)) {
                return false; // empty exponent
            }
            int n = 0;
            more = p != end;
            while (more && is_digit(*p)) {
                if (e10 > 2147483647 / 10) return false;
                e10 = e10 * 10 + (int)(*p - '0');
                ++p;
                ++n;
                more = p != end;
            }
            e10 *= (esign == '+' ? 1 : -1);
            if (n == 0) return false;
        }
    }
    *out = (sign == '+' ? 1 : -1) * (e10 ? std::ldexp(m * std::pow(5.0, e10), e10) : m);
    return true;
}

// parseReal: skip blanks, parse up to the next blank/CR, narrow to float.
float parse_real(const char** tok, double dflt) {
    *tok += std::strspn(*tok, " \t");
    const char* end = *tok + std::strcspn(*tok, " \t\r");
    double v = dflt;
    parse_double(*tok, end, &v);
    *tok = end;
    return (float)v;
}

// fixIndex: 1-based or negative-relative.
bool fix_index(int idx, int n, int* ret, bool allow_zero) {
    if (idx > 0) {
        *ret = idx - 1;
        return true;
    }
    if (idx == 0) {
        *ret = -1;
        return allow_zero;
    }
    *ret = n + idx;
    return *ret >= 0;
}

// parseTriple: `v`, `v/vt`, `v//vn`, `v/vt/vn`; only the vertex index is kept.
bool parse_corner(const char** tok, int nv, int nvn, int nvt, int* vi) {
    int dummy;
    if (!fix_index(std::atoi(*tok), nv, vi, false)) return false;
    *tok += std::strcspn(*tok, "/ \t\r");
    if ((*tok)[0] != '/') return true;
    ++*tok;
    if ((*tok)[0] == '/') { // v//vn
        ++*tok;
        if (!fix_index(std::atoi(*tok), nvn, &dummy, true)) return false;
        *tok += std::strcspn(*tok, "/ \t\r");
        return true;
    }
    if (!fix_index(std::atoi(*tok), nvt, &dummy, true)) return false; // v/vt
    *tok += std::strcspn(*tok, "/ \t\r");
    if ((*tok)[0] != '/') return true;
    ++*tok; // v/vt/vn
    if (!fix_index(std::atoi(*tok), nvn, &dummy, true)) return false;
    *tok += std::strcspn(*tok, "/ \t\r");
    return true;
}

// Point-in-triangle test of the ear clipper (W. Randolph Franklin's pnpoly, float).
bool pnpoly3(const float* vx, const float* vy, float tx, float ty) {
    bool c = false;
    for (int i = 0, j = 2; i < 3; j = i++) {
        if (((vy[i] > ty) != (vy[j] > ty)) &&
            (tx < (vx[j] - vx[i]) * (ty - vy[i]) / (vy[j] - vy[i]) + vx[i]))
            c = !c;
    }
    return c;
}

void emit(std::vector<uint32_t>& out, int a, int b, int c) {
    out.push_back((uint32_t)a);
    out.push_back((uint32_t)b);
    out.push_back((uint32_t)c);
}

// Triangulates one face (vertex indices `f`) the way exportGroupsToShape does.
void triangulate(const std::vector<int>& f, const std::vector<float>& v, std::vector<uint32_t>& out) {
    const size_t n = f.size();
    if (n < 3) return; // degenerate face
    if (n == 3) {
        emit(out, f[0], f[1], f[2]);
        return;
    }
    auto valid = [&](int vi) { return (3 * (size_t)vi + 2) < v.size(); };
    if (n == 4) {
        if (!valid(f[0]) || !valid(f[1]) || !valid(f[2]) || !valid(f[3])) return;
        const float* p0 = &v[3 * (size_t)f[0]];
        const float* p1 = &v[3 * (size_t)f[1]];
        const float* p2 = &v[3 * (size_t)f[2]];
        const float* p3 = &v[3 * (size_t)f[3]];
        float ax = p2[0] - p0[0], ay = p2[1] - p0[1], az = p2[2] - p0[2];
        float bx = p3[0] - p1[0], by = p3[1] - p1[1], bz = p3[2] - p1[2];
        float s02 = ax * ax + ay * ay + az * az;
        float s13 = bx * bx + by * by + bz * bz;
        if (s02 < s13) {
            emit(out, f[0], f[1], f[2]);
            emit(out, f[0], f[2], f[3]);
        } else {
            emit(out, f[0], f[1], f[3]);
            emit(out, f[1], f[2], f[3]);
        }
        return;
    }
    // Ear clipping.  Pick the projection plane from the first corner with a non-zero cross.
    size_t axes[2] = {1, 2};
    for (size_t k = 0; k < n; ++k) {
        int i0 = f[k % n], i1 = f[(k + 1) % n], i2 = f[(k + 2) % n];
        if (!valid(i0) || !valid(i1) || !valid(i2)) continue;
        const float* a = &v[3 * (size_t)i0];
        const float* b = &v[3 * (size_t)i1];
        const float* c = &v[3 * (size_t)i2];
        float e0x = b[0] - a[0], e0y = b[1] - a[1], e0z = b[2] - a[2];
        float e1x = c[0] - b[0], e1y = c[1] - b[1], e1z = c[2] - b[2];
        float cx = std::fabs(e0y * e1z - e0z * e1y);
        float cy = std::fabs(e0z * e1x - e0x * e1z);
        float cz = std::fabs(e0x * e1y - e0y * e1x);
        const float eps = std::numeric_limits<float>::epsilon();
        if (cx > eps || cy > eps || cz > eps) {
            if (!(cx > cy && cx > cz)) {
                axes[0] = 0;
                if (cz > cx && cz > cy) axes[1] = 1;
            }
            break;
        }
    }
    std::vector<int> rem = f;
    size_t guess = 0;
    size_t iters_left = n;
    size_t prev_size = rem.size();
    float vx[3], vy[3];
    int ind[3];
    while (rem.size() > 3 && iters_left > 0) {
        const size_t m = rem.size();
        if (guess >= m) guess -= m;
        if (prev_size != m) {
            prev_size = m;
            iters_left = m;
        } else {
            --iters_left;
        }
        for (int k = 0; k < 3; ++k) {
            ind[k] = rem[(guess + (size_t)k) % m];
            size_t vi = (size_t)ind[k];
            if ((vi * 3 + axes[0]) >= v.size() || (vi * 3 + axes[1]) >= v.size()) {
                vx[k] = 0.0f;
                vy[k] = 0.0f;
            } else {
                vx[k] = v[vi * 3 + axes[0]];
                vy[k] = v[vi * 3 + axes[1]];
            }
        }
        float e0x = vx[1] - vx[0], e0y = vy[1] - vy[0];
        float e1x = vx[2] - vx[1], e1y = vy[2] - vy[1];
        float cross = e0x * e1y - e0y * e1x;
        float area = (vx[0] * vy[1] - vy[0] * vx[1]) * 0.5f;
        if (cross * area < 0.0f) { // reflex corner
            guess += 1;
            continue;
        }
        bool overlap = false;
        for (size_t o = 3; o < m; ++o) {
            size_t idx = (guess + o) % m;
            if (idx >= rem.size()) continue;
            size_t ovi = (size_t)rem[idx];
            if ((ovi * 3 + axes[0]) >= v.size() || (ovi * 3 + axes[1]) >= v.size()) continue;
            if (pnpoly3(vx, vy, v[ovi * 3 + axes[0]], v[ovi * 3 + axes[1]])) {
                overlap = true;
                break;
            }
        }
        if (overlap) {
            guess += 1;
            continue;
        }
        emit(out, ind[0], ind[1], ind[2]);
        // remove the ear tip (guess + 1)
        rem.erase(rem.begin() + (long)((guess + 1) % m));
    }
    if (rem.size() == 3) emit(out, rem[0], rem[1], rem[2]);
}

} // namespace

int obj_load_triangles(const char* path, std::vector<float>& pos, std::vector<uint32_t>& idx,
                       std::string& err) {
    std::ifstream in(path, std::ios::binary);
    if (!in) {
        err = std::string("cannot open OBJ file: ") + path;
        return TRT_ERR_IO;
    }
    pos.clear();
    idx.clear();
    int nvn = 0, nvt = 0;
    std::string line;
    size_t line_no = 0;
    std::vector<int> face;
    while (std::getline(in, line)) {
        ++line_no;
        if (!line.empty() && line.back() == '\r') line.pop_back();
        const char* t = line.c_str();
        t += std::strspn(t, " \t");
        if (t[0] == '\0' || t[0] == '#') continue;
        if (t[0] == 'v' && is_space(t[1])) {
            t += 2;
            float x = parse_real(&t, 0.0), y = parse_real(&t, 0.0), z = parse_real(&t, 0.0);
            pos.push_back(x);
            pos.push_back(y);
            pos.push_back(z);
            continue;
        }
        if (t[0] == 'v' && t[1] == 'n' && is_space(t[2])) {
            ++nvn;
            continue;
        }
        if (t[0] == 'v' && t[1] == 't' && is_space(t[2])) {
            ++nvt;
            continue;
        }
        if (t[0] == 'f' && is_space(t[1])) {
            t += 2;
            t += std::strspn(t, " \t");
            face.clear();
            while (!is_eol(t[0]) && t[0] != '#') {
                int vi;
                if (!parse_corner(&t, (int)(pos.size() / 3), nvn, nvt, &vi)) {
                    err = std::string(path) + ":" + std::to_string(line_no) +
                          ": invalid face vertex index";
                    return TRT_ERR_IO;
                }
                face.push_back(vi);
                t += std::strspn(t, " \t\r");
            }
            triangulate(face, pos, idx);
            continue;
        }
        // o, g, s, usemtl, mtllib, l, p, vw ...: no effect on the triangle list
    }
    return TRT_OK;
}

} // namespace trt
