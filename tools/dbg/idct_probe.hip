// Debug probe: runs jpeg_kernel.hip's idct_kernel on blocks with one non-zero coefficient and
// prints the 8x8 outputs (compare with oracle/jpeg_ref.idct_planes).
#include "../../vkcomputeshader_tinyraytracer_amd/csrc/jpeg_kernel.hip"
#include <cstdio>
int main() {
    using namespace trt::jpeg;
    const int nb = 4;
    std::vector<int16_t> coef(64 * nb, 0);
    coef[0 * 64 + 0] = 10;   // DC
    coef[1 * 64 + 1] = 20;   // (0,1)
    coef[2 * 64 + 8] = 20;   // (1,0)
    coef[3 * 64 + 2] = 20;   // (0,2)
    std::vector<uint16_t> q(64, 1);
    int16_t* dc; uint16_t* dq; uint8_t* ds;
    hipMalloc(&dc, coef.size() * 2); hipMalloc(&dq, 128); hipMalloc(&ds, 64 * nb);
    hipMemcpy(dc, coef.data(), coef.size() * 2, hipMemcpyHostToDevice);
    hipMemcpy(dq, q.data(), 128, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(idct_kernel, dim3(1), dim3(256), 0, 0, dc, dq, ds, (uint32_t)nb, (uint32_t)nb, (uint32_t)(8 * nb));
    std::vector<uint8_t> out(64 * nb);
    hipMemcpy(out.data(), ds, out.size(), hipMemcpyDeviceToHost);
    for (int b = 0; b < nb; ++b) {
        printf("block %d\n", b);
        for (int r = 0; r < 8; ++r) {
            for (int c = 0; c < 8; ++c) printf("%4d", out[r * 8 * nb + 8 * b + c]);
            printf("\n");
        }
    }
    return 0;
}
