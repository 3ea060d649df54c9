// Diagnostic: which SIMD each wave of a resident workgroup lands on, and the
// workgroup's LDS base (HW_REG_HW_ID / HW_REG_LDS_ALLOC).  256-thread
// workgroups with 52 KB of LDS, 768 of them, as the c2 solver launch.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
__global__ void probe(unsigned* out, int spin) {
    extern __shared__ double lds[];
    const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | (0 << 6) | 4);
    const unsigned la = __builtin_amdgcn_s_getreg((31 << 11) | (0 << 6) | 6);
    if ((threadIdx.x & 63) == 0) {
        out[(blockIdx.x * 4 + (threadIdx.x >> 6)) * 2] = hw;
        out[(blockIdx.x * 4 + (threadIdx.x >> 6)) * 2 + 1] = la;
    }
    double a = threadIdx.x;
    for (int i = 0; i < spin; ++i) a = a * 0.999 + 1.0;
    lds[threadIdx.x] = a;
    __syncthreads();
    if (a == -1.0) out[0] = (unsigned)lds[(threadIdx.x + 1) & 255];
}
int main() {
    const int G = 768;
    unsigned* d;
    hipMalloc(&d, G * 4 * 2 * sizeof(unsigned));
    hipLaunchKernelGGL(probe, dim3(G), dim3(256), 51952, 0, d, 200000);
    std::vector<unsigned> h(G * 8);
    hipMemcpy(h.data(), d, h.size() * 4, hipMemcpyDeviceToHost);
    int hist[4][4] = {};
    for (int b = 0; b < G; ++b) {
        unsigned s0 = (h[b * 8] >> 4) & 3;
        for (int w = 0; w < 4; ++w) hist[w][(h[(b * 4 + w) * 2] >> 4) & 3]++;
        if (b < 24) {
            printf("wg %3d:", b);
            for (int w = 0; w < 4; ++w) {
                unsigned hw = h[(b * 4 + w) * 2], la = h[(b * 4 + w) * 2 + 1];
                printf("  w%d simd %u wave %2u cu %2u se %u lds_base %3u", w, (hw >> 4) & 3, hw & 15,
                       (hw >> 8) & 15, (hw >> 13) & 7, la & 0xff);
            }
            printf("\n");
            (void)s0;
        }
    }
    for (int w = 0; w < 4; ++w)
        printf("wave %d simd histogram: %d %d %d %d\n", w, hist[w][0], hist[w][1], hist[w][2], hist[w][3]);
    return 0;
}
