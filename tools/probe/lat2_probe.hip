// More dependent-chain latencies on gfx950 (one workgroup of 256 threads): lane swaps
// (v_permlane16_swap / v_permlane32_swap), an LDS load whose address depends on the
// previous load, a workgroup barrier (4 waves), and s_memtime ticks per s_memrealtime
// tick (100 MHz) to convert.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/probe/lat2_probe.hip -o tools/probe/lat2_probe
#include <hip/hip_runtime.h>
#include <stdio.h>

__device__ __forceinline__ double sw32(double v) {
    const long long b = __double_as_longlong(v);
    const auto lo = __builtin_amdgcn_permlane32_swap((unsigned)b, (unsigned)b, false, false);
    const auto hi = __builtin_amdgcn_permlane32_swap((unsigned)(b >> 32), (unsigned)(b >> 32), false, false);
    return __longlong_as_double(((long long)hi[1] << 32) | lo[1]);
}
__device__ __forceinline__ double sw16(double v) {
    const long long b = __double_as_longlong(v);
    const auto lo = __builtin_amdgcn_permlane16_swap((unsigned)b, (unsigned)b, false, false);
    const auto hi = __builtin_amdgcn_permlane16_swap((unsigned)(b >> 32), (unsigned)(b >> 32), false, false);
    return __longlong_as_double(((long long)hi[1] << 32) | lo[1]);
}

__global__ __launch_bounds__(256) void lat(long long* out, double* sink, int n) {
    __shared__ double sh[1024];
    __shared__ int ish[1024];
    const int t = threadIdx.x, lane = t & 63;
    for (int i = t; i < 1024; i += 256) {
        sh[i] = 1.0 + i * 1e-9;
        ish[i] = (i * 37 + 11) & 1023;
    }
    __syncthreads();
    double a = 1.0 + lane * 1e-9;
    long long r0 = __builtin_amdgcn_s_memrealtime(), m0 = __builtin_amdgcn_s_memtime();
    long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 1
    for (int i = 0; i < n; ++i) {
#pragma unroll
        for (int k = 0; k < 8; ++k) a = sw32(a) * 0.999999;
    }
    long long t1 = __builtin_amdgcn_s_memtime();
#pragma unroll 1
    for (int i = 0; i < n; ++i) {
#pragma unroll
        for (int k = 0; k < 8; ++k) a = sw16(a) * 0.999999;
    }
    long long t2 = __builtin_amdgcn_s_memtime();
    int idx = lane;
#pragma unroll 1
    for (int i = 0; i < n; ++i) {
#pragma unroll
        for (int k = 0; k < 8; ++k) idx = ish[idx];
    }
    long long t3 = __builtin_amdgcn_s_memtime();
    double acc = 0.0;
#pragma unroll 1
    for (int i = 0; i < n; ++i) {
#pragma unroll
        for (int k = 0; k < 8; ++k) acc += sh[(idx + k * 8) & 1023];   // independent loads
    }
    long long t4 = __builtin_amdgcn_s_memtime();
#pragma unroll 1
    for (int i = 0; i < n; ++i) {
#pragma unroll
        for (int k = 0; k < 8; ++k) __syncthreads();
    }
    long long t5 = __builtin_amdgcn_s_memtime();
#pragma unroll 1
    for (int i = 0; i < n; ++i) {
#pragma unroll
        for (int k = 0; k < 8; ++k) __builtin_amdgcn_s_barrier();
    }
    long long t6 = __builtin_amdgcn_s_memtime();
    long long r1 = __builtin_amdgcn_s_memrealtime(), m1 = __builtin_amdgcn_s_memtime();
    sink[t] = a + idx + acc;
    if (t == 0) {
        out[0] = t1 - t0; out[1] = t2 - t1; out[2] = t3 - t2; out[3] = t4 - t3; out[4] = t5 - t4;
        out[5] = t6 - t5; out[6] = r1 - r0; out[7] = m1 - m0;
    }
}

int main() {
    long long* d; double* s;
    (void)hipMalloc(&d, 64 * 8); (void)hipMalloc(&s, 256 * 8);
    const int n = 500;
    hipLaunchKernelGGL(lat, dim3(1), dim3(256), 0, 0, d, s, n);
    (void)hipDeviceSynchronize();
    hipLaunchKernelGGL(lat, dim3(1), dim3(256), 0, 0, d, s, n);
    if (hipDeviceSynchronize() != hipSuccess) { printf("failed\n"); return 1; }
    long long h[8];
    (void)hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
    const double links = 8.0 * n;
    printf("s_memtime ticks per 100 MHz realtime tick: %.2f (-> %.0f MHz)\n", (double)h[7] / h[6], 100.0 * h[7] / h[6]);
    printf("permlane32_swap x2 + mul chain   %6.1f cycles/link\n", h[0] / links);
    printf("permlane16_swap x2 + mul chain   %6.1f cycles/link\n", h[1] / links);
    printf("ds_read_b32 pointer chase        %6.1f cycles/link\n", h[2] / links);
    printf("ds_read_b64 independent (8/grp)  %6.1f cycles/load\n", h[3] / links);
    printf("__syncthreads (256 threads)      %6.1f cycles each\n", h[4] / links);
    printf("s_barrier (256 threads)          %6.1f cycles each\n", h[5] / links);
    return 0;
}
