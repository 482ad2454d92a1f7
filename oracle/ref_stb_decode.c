/* TEST INFRASTRUCTURE ONLY — golden generator compiled against the reference's own vendored
 * stb_image v2.22 (/root/reference/VulkanComputeShaderApplication/lib/stb_image.h, included
 * in place, never copied).  Built into oracle/_ref/ by `make -C oracle ref`.
 *
 * For each JPEG on the command line it calls stbi_load(path, &w, &h, &n, STBI_rgb_alpha) —
 * the reference's call for the envmap (main.cpp:930) — and writes the RGBA8 buffer to
 * <out> (raw bytes) and "w h n" to stdout.  Default compiler flags on x86-64 select stb's
 * SSE2 IDCT / colour / upsampling kernels, as the reference's x64 build does.
 */
#define STB_IMAGE_IMPLEMENTATION
#define STBI_ONLY_JPEG
#include "stb_image.h"

#include <stdio.h>

int main(int argc, char** argv) {
    if (argc < 3 || (argc - 1) % 2) {
        fprintf(stderr, "usage: %s in.jpg out.rgba [in.jpg out.rgba ...]\n", argv[0]);
        return 2;
    }
    for (int a = 1; a + 1 < argc; a += 2) {
        int w, h, n;
        unsigned char* px = stbi_load(argv[a], &w, &h, &n, STBI_rgb_alpha);
        if (!px) {
            fprintf(stderr, "stbi_load failed for %s: %s\n", argv[a], stbi_failure_reason());
            return 1;
        }
        FILE* f = fopen(argv[a + 1], "wb");
        if (!f || fwrite(px, 1, (size_t)w * h * 4, f) != (size_t)w * h * 4) return 1;
        fclose(f);
        printf("%d %d %d\n", w, h, n);
        stbi_image_free(px);
    }
    return 0;
}
