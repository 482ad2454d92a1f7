// TEST INFRASTRUCTURE ONLY — golden generator compiled against the reference's own vendored
// tinyobjloader (/root/reference/VulkanComputeShaderApplication/lib/tiny_obj_loader.h,
// included in place, never copied).  Built into oracle/_ref/ by `make -C oracle ref`.
//
// For each OBJ given on the command line it calls tinyobj::LoadObj with the reference's
// arguments (main.cpp:2292-2300: default triangulate = true) and walks the shapes exactly as
// loadObjAsTriangles does (main.cpp:2302-2332, including its `fv != 3` skip), writing
//   <out>.pos : float32 xyz of attrib.vertices
//   <out>.idx : uint32 vertex_index triples of the triangles loadObjAsTriangles keeps
#define TINYOBJLOADER_IMPLEMENTATION
#include "tiny_obj_loader.h"

#include <cstdio>
#include <string>
#include <vector>

int main(int argc, char** argv) {
    if (argc < 3 || (argc - 1) % 2) {
        std::fprintf(stderr, "usage: %s in.obj out_prefix [in.obj out_prefix ...]\n", argv[0]);
        return 2;
    }
    for (int a = 1; a + 1 < argc; a += 2) {
        tinyobj::attrib_t attrib;
        std::vector<tinyobj::shape_t> shapes;
        std::vector<tinyobj::material_t> materials;
        std::string warn, err;
        if (!tinyobj::LoadObj(&attrib, &shapes, &materials, &warn, &err, argv[a])) {
            std::fprintf(stderr, "LoadObj failed for %s: %s%s\n", argv[a], warn.c_str(), err.c_str());
            return 1;
        }
        std::vector<uint32_t> idx;
        for (const auto& shape : shapes) {
            size_t index_offset = 0;
            for (size_t f = 0; f < shape.mesh.num_face_vertices.size(); f++) {
                int fv = shape.mesh.num_face_vertices[f];
                if (fv != 3) continue;
                for (int i = 0; i < 3; i++)
                    idx.push_back((uint32_t)shape.mesh.indices[index_offset + i].vertex_index);
                index_offset += fv;
            }
        }
        std::string pre = argv[a + 1];
        FILE* fp = std::fopen((pre + ".pos").c_str(), "wb");
        FILE* fi = std::fopen((pre + ".idx").c_str(), "wb");
        if (!fp || !fi) return 1;
        std::fwrite(attrib.vertices.data(), sizeof(float), attrib.vertices.size(), fp);
        std::fwrite(idx.data(), sizeof(uint32_t), idx.size(), fi);
        std::fclose(fp);
        std::fclose(fi);
        std::printf("%s: %zu vertices, %zu triangles\n", argv[a], attrib.vertices.size() / 3, idx.size() / 3);
    }
    return 0;
}
