// Micro-benchmark: the row-by-row triangular solve (Solver) against the blocked solve
// with inverted 4 x 4 / 8 x 8 diagonal blocks (BSolver), n compile-time as in the c2
// kernel (81) and c5's Hp 30 (121).  One workgroup alone, 1 and 2 per CU.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include tools/probe/bsolve_probe.hip -o tools/probe/bsolve_probe
#define SCPQP_DIAG_NO_HOST
#include "../../senquential-convex-programming-for-trajectory-planning_amd/csrc/scpqp.hip"

#include <vector>

namespace {
template <int VAR, int NC>
__global__ __launch_bounds__(256, 2) void probe(double* xout, long long* cyc, int reps) {
    constexpr int n = NC;
    constexpr int R = (n + 63) / 64;
    ldouble* H = (ldouble*)smem_;
    const int hsz = pad2(roff(n + 1) + 16);
    ldouble* dinv = H + hsz;
    ldouble* b = dinv + pad2(n);
    ldouble* x = b + pad2(n);
    for (int e = threadIdx.x; e < hsz; e += 256) H[e] = 0.0;
    __syncthreads();
    for (int i = threadIdx.x; i < n; i += 256) {
        for (int j = 0; j < i; ++j) H[roff(i) + j] = 0.3 * sin(0.7 * i + 1.3 * j) / (1.0 + 0.05 * (i - j));
        H[roff(i) + i] = 1.0;
        dinv[i] = 1.0 / (1.0 + 0.01 * i);
        b[i] = cos(0.37 * i);
    }
    __syncthreads();
    if (VAR == 1) block_inverses<4>(H, n);
    if (VAR == 2) block_inverses<8>(H, n);
    __syncthreads();
    if (wave_id() == 0) {
        const long long t0 = __builtin_amdgcn_s_memtime();
        for (int r = 0; r < reps; ++r) {
            if constexpr (VAR == 0) {
                Solver<R, ldouble*, 4> S(H, dinv, n, 0, b);
                S.run(x);
            } else if constexpr (VAR == 1) {
                BSolver<R, 4, ldouble*> S(H, dinv, n, b);
                S.run(x);
            } else {
                BSolver<R, 8, ldouble*> S(H, dinv, n, b);
                S.run(x);
            }
            __builtin_amdgcn_s_waitcnt(0);
        }
        const long long t1 = __builtin_amdgcn_s_memtime();
        if ((threadIdx.x & 63) == 0) cyc[blockIdx.x] = t1 - t0;
    }
    __syncthreads();
    if (blockIdx.x == 0)
        for (int i = threadIdx.x; i < n; i += 256) xout[i] = x[i];
}
}  // namespace

template <int VAR, int NC>
void run(const char* name, int grid, int reps, double* dx, long long* dc, const double* ref) {
    constexpr int n = NC;
    const size_t lds = (size_t)(pad2(roff(n + 1) + 16) + 3 * pad2(n)) * 8;
    auto k = probe<VAR, NC>;
    (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipLaunchKernelGGL(k, dim3(grid), dim3(256), lds, 0, dx, dc, reps);
    (void)hipDeviceSynchronize();
    std::vector<long long> c(grid);
    std::vector<double> x(n);
    (void)hipMemcpy(c.data(), dc, grid * 8, hipMemcpyDeviceToHost);
    (void)hipMemcpy(x.data(), dx, n * 8, hipMemcpyDeviceToHost);
    double mx = 0, err = 0;
    for (int g = 0; g < grid; ++g) mx = c[g] > mx ? c[g] : mx;
    for (int i = 0; i < n; ++i) err = fmax(err, fabs(x[i] - ref[i]));
    printf("%-16s n=%3d grid=%4d: %8.0f cycles/solve (max over WGs), |x - ref| %.1e\n", name, n, grid,
           mx / reps, err);
}

template <int NC>
void all(double* dx, long long* dc) {
    constexpr int n = NC;
    std::vector<double> L(n * n, 0.0), bb(n), y(n), xr(n);
    for (int i = 0; i < n; ++i) {
        for (int j = 0; j < i; ++j) L[i * n + j] = 0.3 * sin(0.7 * i + 1.3 * j) / (1.0 + 0.05 * (i - j));
        bb[i] = cos(0.37 * i);
    }
    for (int i = 0; i < n; ++i) { double s = bb[i]; for (int j = 0; j < i; ++j) s -= L[i * n + j] * y[j]; y[i] = s; }
    for (int i = 0; i < n; ++i) y[i] *= 1.0 / (1.0 + 0.01 * i);
    for (int i = n - 1; i >= 0; --i) { double s = y[i]; for (int j = i + 1; j < n; ++j) s -= L[j * n + i] * xr[j]; xr[i] = s; }
    for (int grid : {1, 256, 512}) {
        run<0, NC>("Solver", grid, 50, dx, dc, xr.data());
        run<1, NC>("BSolver<4>", grid, 50, dx, dc, xr.data());
        run<2, NC>("BSolver<8>", grid, 50, dx, dc, xr.data());
    }
}

int main() {
    double* dx;
    long long* dc;
    (void)hipMalloc(&dx, 512 * 8);
    (void)hipMalloc(&dc, 2048 * 8);
    all<81>(dx, dc);
    all<121>(dx, dc);
    return 0;
}
