// tests/native/drop_in_host.cpp — a C++ host of the C-ABI with no Python and no torch in the
// process: the reference's own caller (ComputeShaderApplication::createShaderStorageBuffers,
// main.cpp:1494-1664, and drawFrame, main.cpp:2165-2205) with its Vulkan compute objects replaced
// by libtrt, as INTEGRATION.md §2 shows.  libtrt and this program resolve the HIP runtime and RCCL
// through their RUNPATH (/opt/rocm/lib), not through a Python process's already-loaded copies.
//
// usage:
//   drop_in_host <mesh_dump> <out_dir>     render the frames below; one raw RGBA8 file per frame
//                                          (<out_dir>/<name>.rgba) and one JSON line per frame
//   drop_in_host --envmap W H <out_file>   write the synthetic envmap (no GPU; checks the port)
//   drop_in_host --bench <mesh_dump> <frames> [in_flight]
//                                          time the shipped frame along the camera walk through
//                                          the C-ABI with this process's environment (bench.py
//                                          runs it with GPU_MAX_HW_QUEUES unset, as the reference's
//                                          own host would start): `frames` frames in one
//                                          trt_render_frames call (auto in-flight count, or
//                                          `in_flight`), then the drawFrame pacing (trt_render into
//                                          host memory, one call per frame); one JSON line
//
// Frames (1024x768):
//   shipped          the shipped frame: glass + whisky + ice (config.hpp:97-101) from the mesh
//                    dump through trt_scene_add_mesh, depth 20, reference flags, trt_render
//                    into host memory (the drawFrame binding of INTEGRATION.md §2)
//   shipped_walk_k   k = 0..3: the same scene along the camera walk of processInput
//                    (main.cpp:391-403) in one trt_render_frames call into device memory
//   c2_walk_k        k = 0..7: 4 spheres + floor + envmap, depth 4, no triangles (ntri = 0), one
//                    trt_render_frames call (multi-frame launches)
//   multi_c2         the C2 frame through trt_multi_create / trt_multi_upload_scene /
//                    trt_render_multi on a one-device communicator, host output
#include <hip/hip_runtime.h>

#include <cerrno>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <stdexcept>
#include <string>
#include <vector>

#include "trt/abi.h"

namespace {

[[noreturn]] void die(const std::string& msg) {
    std::fprintf(stderr, "drop_in_host: %s\n", msg.c_str());
    std::exit(1);
}

void check(int rc, const char* what, const trt_ctx* ctx = nullptr) {
    if (rc != TRT_OK) die(std::string(what) + " failed (" + std::to_string(rc) + "): " + (ctx ? trt_last_error(ctx) : ""));
}

void hcheck(hipError_t e, const char* what) {
    if (e != hipSuccess) die(std::string(what) + ": " + hipGetErrorString(e));
}

trt_vec4 v4(float x, float y, float z, float w) { return trt_vec4{x, y, z, w}; }

trt_material material(trt_vec4 albedo, trt_vec4 ds, float ior) {
    return trt_material{albedo, ds, v4(ior, 0, 0, 0)};
}

// main.cpp:125-128 sphere materials
const trt_material IVORY = material(v4(0.9f, 0.5f, 0.1f, 0.0f), v4(0.4f, 0.4f, 0.3f, 50.0f), 1.0f);
const trt_material GLASS = material(v4(0.0f, 0.9f, 0.1f, 0.8f), v4(0.6f, 0.7f, 0.8f, 125.0f), 1.5f);
const trt_material RED_RUBBER = material(v4(1.4f, 0.3f, 0.0f, 0.0f), v4(0.3f, 0.1f, 0.1f, 10.0f), 1.0f);
const trt_material MIRROR = material(v4(0.0f, 16.0f, 0.8f, 0.0f), v4(1.0f, 1.0f, 1.0f, 1425.0f), 1.0f);

// updateUniformBuffer (main.cpp:2165-2179): spheres main.cpp:132-137, lights :139-143
trt_ubo make_ubo(float cx, float cy, float cz) {
    trt_ubo u;
    std::memset(&u, 0, sizeof(u));
    u.sphere0 = trt_sphere{v4(-3.0f, 0.0f, -16.0f, 2.0f), IVORY};
    u.sphere1 = trt_sphere{v4(-1.0f, -1.5f, -12.0f, 2.0f), GLASS};
    u.sphere2 = trt_sphere{v4(1.5f, -0.5f, -18.0f, 3.0f), RED_RUBBER};
    u.sphere3 = trt_sphere{v4(7.0f, 5.0f, -18.0f, 4.0f), MIRROR};
    u.light0 = v4(-20.0f, 20.0f, 20.0f, 1.0f);
    u.light1 = v4(30.0f, 50.0f, -25.0f, 1.0f);
    u.light2 = v4(30.0f, 20.0f, 30.0f, 1.0f);
    u.camPos = v4(cx, cy, cz, 1.0f);
    const float fmax = 3.402823466e38f;
    u.bboxMin = v4(fmax, fmax, fmax, fmax);
    u.bboxMax = v4(-fmax, -fmax, -fmax, -fmax);
    return u;
}

// processInput with W and D held (main.cpp:391-403): cameraPos += speed * (1, 0, -1) per frame
std::vector<trt_ubo> camera_walk(uint32_t n, float speed = 0.02f) {
    std::vector<trt_ubo> v;
    for (uint32_t k = 0; k < n; ++k) v.push_back(make_ubo(speed * (float)k, 0.0f, speed * -(float)k));
    return v;
}

uint32_t hash32(uint32_t x) {
    const uint32_t state = x * 747796405u + 2891336453u;
    const uint32_t word = ((state >> ((state >> 28u) + 4u)) ^ state) * 277803737u;
    return (word >> 22u) ^ word;
}

// The seeded procedural envmap of the Python package (scene.synthetic_envmap), restated: the
// stand-in for background.jpg (7616x3808, main.cpp:928-949).
std::vector<uint8_t> synthetic_envmap(uint32_t W, uint32_t H, uint32_t seed = 0) {
    std::vector<uint8_t> out((size_t)W * H * 4);
    std::vector<uint32_t> hx(W);
    for (uint32_t x = 0; x < W; ++x) hx[x] = hash32(x ^ (uint32_t)(seed * 0x9E3779B9u));
    auto clip8 = [](double v) -> uint8_t { return (uint8_t)(v < 0 ? 0.0 : v > 255 ? 255.0 : v); };
    for (uint32_t y = 0; y < H; ++y) {
        const float v = ((float)y + 0.5f) / (float)H;
        const bool sky = v < 0.5f;
        const float t = std::fabs(v - 0.5f) * 2.0f;
        const float r0 = sky ? 120.0f + 100.0f * t : 90.0f - 40.0f * t;
        const float g0 = sky ? 170.0f + 60.0f * t : 70.0f - 30.0f * t;
        const float b0 = sky ? 230.0f - 20.0f * t : 50.0f - 20.0f * t;
        const bool grid_y = (y % 256u) < 6u;
        for (uint32_t x = 0; x < W; ++x) {
            const uint32_t n = hash32(hx[x] + y * 0x85EBCA6Bu);
            const int32_t noise = (int32_t)(n & 31u) - 16;
            const bool grid = grid_y || (x % 256u) < 6u;
            uint8_t* px = &out[((size_t)y * W + x) * 4];
            px[0] = clip8((double)(grid ? 250.0f : r0) + noise);
            px[1] = clip8((double)(grid ? 240.0f : g0) + ((noise * 3) >> 2));
            px[2] = clip8((double)(grid ? 200.0f : b0) + (noise >> 1));
            px[3] = 255;
        }
    }
    return out;
}

struct Mesh {
    std::string name;
    std::vector<float> pos;
    std::vector<uint32_t> idx;
};

// tests/golden/dropin_meshes.bin (tests/golden/make_dropin_dump.py): "TRTMESH1", u32 count, then
// per mesh u32 name length, name, u32 nverts, u32 ntris, float pos[3 nverts], u32 idx[3 ntris]
std::vector<Mesh> read_dump(const std::string& path) {
    std::ifstream f(path, std::ios::binary);
    if (!f) die("cannot open " + path);
    char magic[8];
    f.read(magic, 8);
    if (!f || std::memcmp(magic, "TRTMESH1", 8) != 0) die("bad mesh dump " + path);
    auto u32 = [&]() {
        uint32_t v = 0;
        f.read(reinterpret_cast<char*>(&v), 4);
        if (!f) die("truncated mesh dump");
        return v;
    };
    std::vector<Mesh> out(u32());
    for (Mesh& m : out) {
        m.name.resize(u32());
        f.read(&m.name[0], (std::streamsize)m.name.size());
        const uint32_t nv = u32(), nt = u32();
        m.pos.resize((size_t)nv * 3);
        m.idx.resize((size_t)nt * 3);
        f.read(reinterpret_cast<char*>(m.pos.data()), (std::streamsize)(m.pos.size() * 4));
        f.read(reinterpret_cast<char*>(m.idx.data()), (std::streamsize)(m.idx.size() * 4));
        if (!f) die("truncated mesh dump");
    }
    return out;
}

struct ModelInfo {
    const char* asset;
    trt_material mat;
    float scale[3], rotation[3], translation[3];
    int normal_interp;
};

// config.hpp:63-81 (glass / whisky / ice), modelList config.hpp:97-101
const ModelInfo MODEL_LIST[] = {
    {"glass.obj", material(v4(0.0f, 0.3f, 0.05f, 0.9f), v4(0.95f, 0.95f, 0.95f, 80.0f), 1.5f), {1, 1, 1}, {0, 0, 0},
     {0.0f, -2.0f, -8.0f}, 1},
    {"water.obj", material(v4(0.3f, 0.4f, 0.05f, 0.7f), v4(0.9f, 0.6f, 0.3f, 20.0f), 1.2f), {1, 1, 1}, {0, 0, 0},
     {0.0f, -2.0f, -8.0f}, 1},
    {"ice.obj", material(v4(0.05f, 0.4f, 0.2f, 0.8f), v4(0.8f, 0.85f, 0.9f, 20.0f), 1.31f), {1, 1, 1}, {0, 0, 0},
     {0.0f, -2.0f, -8.0f}, 1},
};

void write_frame(const std::string& dir, const std::string& name, const uint8_t* px, size_t bytes) {
    const std::string path = dir + "/" + name + ".rgba";
    FILE* f = std::fopen(path.c_str(), "wb");
    if (!f || std::fwrite(px, 1, bytes, f) != bytes) die("cannot write " + path);
    std::fclose(f);
    std::printf("{\"frame\": \"%s\", \"bytes\": %zu}\n", name.c_str(), bytes);
}

// The shared objects this process actually mapped (the HIP runtime and RCCL it resolved).
void print_runtime() {
    int rt = 0;
    (void)hipRuntimeGetVersion(&rt);
    std::string hip, rccl;
    std::ifstream maps("/proc/self/maps");
    for (std::string line; std::getline(maps, line);) {
        const size_t p = line.find('/');
        if (p == std::string::npos) continue;
        const std::string path = line.substr(p);
        if (hip.empty() && path.find("libamdhip64.so") != std::string::npos) hip = path;
        if (rccl.empty() && path.find("librccl.so") != std::string::npos) rccl = path;
    }
    std::printf("{\"hip_runtime_version\": %d, \"libamdhip64\": \"%s\", \"librccl\": \"%s\", \"trt_version\": \"%s\"}\n",
                rt, hip.c_str(), rccl.c_str(), trt_version());
}

// The shipped scene (config.hpp:97-101) from the mesh dump through the C-ABI builder, uploaded.
void upload_shipped(trt_ctx* ctx, const std::vector<Mesh>& meshes, const std::vector<uint8_t>& env, const trt_ubo& ubo) {
    trt_scene* sb = nullptr;
    check(trt_scene_create(&sb), "trt_scene_create");
    for (const ModelInfo& mi : MODEL_LIST) {
        const Mesh* m = nullptr;
        for (const Mesh& c : meshes)
            if (c.name == mi.asset) m = &c;
        if (!m) die(std::string("mesh dump lacks ") + mi.asset);
        if (trt_scene_add_mesh(sb, m->pos.data(), (uint32_t)(m->pos.size() / 3), m->idx.data(),
                               (uint32_t)(m->idx.size() / 3), &mi.mat, mi.scale, mi.rotation, mi.translation,
                               mi.normal_interp) != TRT_OK)
            die(std::string("trt_scene_add_mesh: ") + trt_scene_last_error(sb));
    }
    std::printf("{\"scene_triangles\": %u, \"scene_batches\": %u}\n", trt_scene_triangle_count(sb),
                trt_scene_model_count(sb));
    check(trt_upload_scene(ctx, &ubo, trt_scene_triangles(sb), trt_scene_triangle_count(sb), trt_scene_models(sb),
                           trt_scene_model_count(sb), env.data(), 7616, 3808),
          "trt_upload_scene", ctx);
    trt_scene_destroy(sb);
}

// --bench: the shipped frame's rate through the C-ABI as a C++ host with its own environment.
int bench(const std::vector<Mesh>& meshes, uint32_t frames, uint32_t in_flight) {
    const std::vector<uint8_t> env = synthetic_envmap(7616, 3808);
    trt_ctx* ctx = nullptr;
    check(trt_create(&ctx, 0), "trt_create");
    const trt_ubo ubo = make_ubo(0, 0, 0);
    upload_shipped(ctx, meshes, env, ubo);
    check(trt_set_frames_in_flight(ctx, in_flight), "trt_set_frames_in_flight", ctx);
    trt_params rp;
    trt_params_default(&rp); // 1024x768, depth 20, reference flags
    const size_t fb = (size_t)rp.width * rp.height * 4;
    uint8_t* dev = nullptr; // one image per frame: the frames of the loop run concurrently
    hcheck(hipMalloc(reinterpret_cast<void**>(&dev), (size_t)frames * fb), "hipMalloc");
    trt_params p = rp;
    p.flags |= TRT_FLAG_DEVICE_PTRS;
    const std::vector<trt_ubo> walk = camera_walk(frames);
    using clk = std::chrono::steady_clock;
    auto run_loop = [&](uint32_t n) { // the first n frames of the walk in one frame-loop call
        check(trt_render_frames(ctx, &p, walk.data(), n, dev, fb, 0), "trt_render_frames", ctx);
        check(trt_synchronize(ctx), "trt_synchronize", ctx);
    };
    run_loop(std::min(frames, 32u)); // warmup: scratch, streams, clocks
    const auto t0 = clk::now();
    run_loop(frames);
    const double loop_ms = std::chrono::duration<double, std::milli>(clk::now() - t0).count();
    // drawFrame pacing: one trt_render per frame into host memory (the INTEGRATION.md binding)
    std::vector<uint8_t> host(fb);
    const uint32_t nd = std::min<uint32_t>(frames, 40);
    for (uint32_t i = 0; i < 4; ++i) check(trt_render(ctx, &rp, host.data(), nullptr, nullptr), "trt_render", ctx);
    const auto t1 = clk::now();
    for (uint32_t i = 0; i < nd; ++i) {
        check(trt_update_ubo(ctx, &walk[i]), "trt_update_ubo", ctx);
        check(trt_render(ctx, &rp, host.data(), nullptr, nullptr), "trt_render", ctx);
    }
    const double draw_ms = std::chrono::duration<double, std::milli>(clk::now() - t1).count();
    const char* q = std::getenv("GPU_MAX_HW_QUEUES");
    std::printf("{\"bench\": \"shipped_frame_c_abi\", \"gpu_max_hw_queues\": \"%s\", \"in_flight_setting\": %u, "
                "\"frames\": %u, \"ms_per_frame\": %.4f, \"fps\": %.1f, \"draw_frame_ms\": %.4f, "
                "\"draw_frames\": %u}\n",
                q ? q : "unset", in_flight, frames, loop_ms / frames, 1000.0 * frames / loop_ms, draw_ms / nd, nd);
    hcheck(hipFree(dev), "hipFree");
    check(trt_destroy(ctx), "trt_destroy");
    return 0;
}

} // namespace

int main(int argc, char** argv) {
    if ((argc == 4 || argc == 5) && std::string(argv[1]) == "--bench")
        return bench(read_dump(argv[2]), (uint32_t)std::strtoul(argv[3], nullptr, 10),
                     argc == 5 ? (uint32_t)std::strtoul(argv[4], nullptr, 10) : 0u);
    if (argc == 5 && std::string(argv[1]) == "--envmap") {
        const uint32_t W = (uint32_t)std::strtoul(argv[2], nullptr, 10), H = (uint32_t)std::strtoul(argv[3], nullptr, 10);
        const std::vector<uint8_t> env = synthetic_envmap(W, H);
        FILE* f = std::fopen(argv[4], "wb");
        if (!f || std::fwrite(env.data(), 1, env.size(), f) != env.size()) die("cannot write envmap");
        std::fclose(f);
        return 0;
    }
    if (argc != 3) die("usage: drop_in_host <mesh_dump> <out_dir> | --envmap W H <out_file>");
    const std::vector<Mesh> meshes = read_dump(argv[1]);
    const std::string out_dir = argv[2];
    const std::vector<uint8_t> env = synthetic_envmap(7616, 3808);

    // createShaderStorageBuffers (main.cpp:1494): the modelList loop through the C-ABI builder
    trt_ctx* ctx = nullptr;
    check(trt_create(&ctx, 0), "trt_create");
    print_runtime();
    const trt_ubo ubo = make_ubo(0, 0, 0);
    upload_shipped(ctx, meshes, env, ubo);

    trt_params rp;
    trt_params_default(&rp); // 1024x768, depth 20, reference flags
    const size_t fb = (size_t)rp.width * rp.height * 4;
    std::vector<uint8_t> host(fb);

    // drawFrame (main.cpp:2181): update the UBO, render, hand the image to the present pass
    check(trt_update_ubo(ctx, &ubo), "trt_update_ubo", ctx);
    check(trt_render(ctx, &rp, host.data(), nullptr, nullptr), "trt_render", ctx);
    write_frame(out_dir, "shipped", host.data(), fb);

    // the mainLoop (main.cpp:405-438) as one frame-loop call, device outputs
    uint8_t* dev = nullptr;
    hcheck(hipMalloc(reinterpret_cast<void**>(&dev), 8 * fb), "hipMalloc");
    {
        const std::vector<trt_ubo> walk = camera_walk(4);
        trt_params p = rp;
        p.flags |= TRT_FLAG_DEVICE_PTRS;
        check(trt_render_frames(ctx, &p, walk.data(), 4, dev, fb, 0), "trt_render_frames (shipped)", ctx);
        check(trt_synchronize(ctx), "trt_synchronize", ctx);
        for (int k = 0; k < 4; ++k) {
            hcheck(hipMemcpy(host.data(), dev + k * fb, fb, hipMemcpyDeviceToHost), "hipMemcpy");
            write_frame(out_dir, "shipped_walk_" + std::to_string(k), host.data(), fb);
        }
    }

    // C2: spheres + floor + envmap, depth 4, no triangles (a scene the reference cannot bind)
    check(trt_upload_scene(ctx, &ubo, nullptr, 0, nullptr, 0, env.data(), 7616, 3808), "trt_upload_scene (C2)", ctx);
    trt_params c2 = rp;
    c2.max_depth = 4;
    c2.flags = TRT_FLAG_SPHERES | TRT_FLAG_FLOOR | TRT_FLAG_ENVMAP | TRT_FLAG_ROW_QUIRK;
    {
        const std::vector<trt_ubo> walk = camera_walk(8);
        trt_params p = c2;
        p.flags |= TRT_FLAG_DEVICE_PTRS;
        check(trt_render_frames(ctx, &p, walk.data(), 8, dev, fb, 0), "trt_render_frames (C2)", ctx);
        check(trt_synchronize(ctx), "trt_synchronize", ctx);
        for (int k = 0; k < 8; ++k) {
            hcheck(hipMemcpy(host.data(), dev + k * fb, fb, hipMemcpyDeviceToHost), "hipMemcpy");
            write_frame(out_dir, "c2_walk_" + std::to_string(k), host.data(), fb);
        }
    }
    hcheck(hipFree(dev), "hipFree");
    check(trt_destroy(ctx), "trt_destroy");

    // the node's GPUs behind the same drawFrame, here a one-device communicator
    trt_multi* m = nullptr;
    const int devs[1] = {0};
    if (trt_multi_create(&m, devs, 1) != TRT_OK) die("trt_multi_create failed");
    if (trt_multi_upload_scene(m, &ubo, nullptr, 0, nullptr, 0, env.data(), 7616, 3808) != TRT_OK)
        die(std::string("trt_multi_upload_scene: ") + trt_multi_last_error(m));
    uint8_t* outs[1] = {host.data()};
    if (trt_render_multi(m, &c2, 8, 0, outs, nullptr) != TRT_OK)
        die(std::string("trt_render_multi: ") + trt_multi_last_error(m));
    write_frame(out_dir, "multi_c2", host.data(), fb);
    trt_multi_destroy(m);
    std::printf("{\"done\": true}\n");
    return 0;
}
