// Micro-benchmark of the L D L' factorisation (device code of
// csrc/scpqp.hip, host side left out): cycles per factorisation of an SPD
// matrix of order n in the packed LDS layout, alone and 3 workgroups per CU.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include tools/probe/chol_probe.hip -o tools/probe/chol_probe
#include "../../senquential-convex-programming-for-trajectory-planning_amd/csrc/scpqp_kernel.h"
#include <vector>

namespace {
template <int R>
struct PLay {
    static constexpr int RMAX = R;
    static constexpr bool HGLOBAL = false;
    static constexpr int OCCV = 3;
    ldouble *H, *dinv, *red;
    int n, lead;
};

template <int VAR, int R>
__global__ __launch_bounds__(256, 3) void chol_probe(double* dout, long long* cyc, int n, int reps) {
    PLay<R> L;
    const int hsz = pad2(roff(n + 1) + 16);
    L.H = (ldouble*)smem_;
    ldouble* K0 = L.H + hsz;
    L.dinv = K0 + hsz;
    L.red = L.dinv + pad2(n);
    L.n = n;
    L.lead = (blockIdx.x % 3) + 1 > 3 ? 0 : (blockIdx.x % 4);
    for (int e = threadIdx.x; e < hsz; e += 256) K0[e] = 0.0;
    __syncthreads();
    // K = n I + S, S_ij = 0.5 sin(i + 2 j) sin(2 i + j) (symmetric): SPD for these n
    for (int i = threadIdx.x; i < n; i += 256)
        for (int j = 0; j <= i; ++j)
            K0[roff(i) + j] = (i == j ? (double)n : 0.0) + 0.5 * sin(0.3 * i + 0.6 * j) * sin(0.6 * i + 0.3 * j);
    __syncthreads();
    long long tot = 0;
    bool ok = true;
    for (int r = 0; r < reps; ++r) {
        for (int e = threadIdx.x; e < hsz; e += 256) L.H[e] = K0[e];
        __syncthreads();
        const long long t0 = __builtin_amdgcn_s_memtime();
        ok = cholesky(L);
        const long long t1 = __builtin_amdgcn_s_memtime();
        tot += t1 - t0;
    }
    if (threadIdx.x == 0) cyc[blockIdx.x] = ok ? tot : -1;
    if (blockIdx.x == 0)
        for (int i = threadIdx.x; i < n; i += 256) dout[i] = L.dinv[i];
}
}  // namespace

template <int VAR, int R>
void run(const char* name, int n, int grid, int reps, double* dd, long long* dc, std::vector<double>& ref) {
    const size_t lds = (size_t)(2 * pad2(roff(n + 1) + 16) + pad2(n) + 128) * 8;
    auto k = chol_probe<VAR, R>;
    (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipLaunchKernelGGL(k, dim3(grid), dim3(256), lds, 0, dd, dc, n, reps);
    (void)hipDeviceSynchronize();
    std::vector<long long> c(grid);
    std::vector<double> d(n);
    (void)hipMemcpy(c.data(), dc, grid * 8, hipMemcpyDeviceToHost);
    (void)hipMemcpy(d.data(), dd, n * 8, hipMemcpyDeviceToHost);
    double mx = 0, err = 0;
    for (int g = 0; g < grid; ++g) mx = c[g] > mx ? c[g] : mx;
    for (int i = 0; i < n; ++i) err = fmax(err, fabs(d[i] - ref[i]) / fabs(ref[i]));
    printf("%-26s n=%3d grid=%4d: %8.0f cycles/factorisation, rel |dinv - ref| %.1e%s\n", name, n, grid,
           mx / reps, err, mx < 0 ? " FAILED" : "");
}

int main() {
    double* dd;
    long long* dc;
    (void)hipMalloc(&dd, 512 * 8);
    (void)hipMalloc(&dc, 2048 * 8);
    for (int n : {81, 121}) {
        std::vector<double> K(n * n), ref(n);
        for (int i = 0; i < n; ++i)
            for (int j = 0; j <= i; ++j)
                K[i * n + j] = K[j * n + i] = (i == j ? (double)n : 0.0) + 0.5 * sin(0.3 * i + 0.6 * j) * sin(0.6 * i + 0.3 * j);
        for (int j = 0; j < n; ++j) {           // host L D L' (right-looking)
            const double D = K[j * n + j];
            ref[j] = 1.0 / D;
            for (int i = j + 1; i < n; ++i) {
                const double l = K[i * n + j] / D;
                for (int k = j + 1; k <= i; ++k) K[i * n + k] -= l * K[k * n + j];
            }
        }
        for (int grid : {1, 768}) {
            const int reps = n > 128 ? 5 : 20;
            if (n <= 128) run<0, 2>("look-ahead L D L'", n, grid, reps, dd, dc, ref);
        }
    }
    return 0;
}
