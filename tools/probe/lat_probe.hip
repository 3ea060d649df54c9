// Dependent-chain latencies on gfx950 (cycles per link, one wave):
// FP64 FMA chain, v_readlane(x2) -> FMA chain, and LDS broadcast read -> FMA.
#include <hip/hip_runtime.h>
#include <stdio.h>

__device__ __forceinline__ double readlane_d(double v, int lane) {
    long long bits = __double_as_longlong(v);
    int lo = __builtin_amdgcn_readlane((int)(bits & 0xffffffffll), lane);
    int hi = __builtin_amdgcn_readlane((int)(bits >> 32), lane);
    return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

__global__ void lat(long long* out, double* sink, int n) {
    __shared__ double sh[256];
    const int lane = threadIdx.x;
    double a = 1.0 + lane * 1e-9, b = 0.999999, c = 1e-7;
    sh[lane] = a;
    __syncthreads();
    long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 1
    for (int i = 0; i < n; ++i) {
#pragma unroll
        for (int k = 0; k < 8; ++k) a = fma(a, b, c);
    }
    long long t1 = __builtin_amdgcn_s_memtime();
#pragma unroll 1
    for (int i = 0; i < n; ++i) {
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const double x = readlane_d(a, (i + k) & 63);
            a = fma(-b, x, a);
        }
    }
    long long t2 = __builtin_amdgcn_s_memtime();
#pragma unroll 1
    for (int i = 0; i < n; ++i) {
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            sh[lane] = a;
            __builtin_amdgcn_s_waitcnt(0);
            const double x = sh[(i + k) & 63];
            a = fma(-b, x, a) * 0.5;
        }
    }
    long long t3 = __builtin_amdgcn_s_memtime();
#pragma unroll 1
    for (int i = 0; i < n; ++i) {
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            a = a * b;   // v_mul_f64
        }
    }
    long long t4 = __builtin_amdgcn_s_memtime();
    double r = __builtin_amdgcn_rcp(a);
#pragma unroll 1
    for (int i = 0; i < n; ++i) {
#pragma unroll
        for (int k = 0; k < 8; ++k) r = __builtin_amdgcn_rcp(r + 1.0);
    }
    long long t5 = __builtin_amdgcn_s_memtime();
    sink[lane] = a + r;
    if (lane == 0) { out[0] = t1 - t0; out[1] = t2 - t1; out[2] = t3 - t2; out[3] = t4 - t3; out[4] = t5 - t4; }
}

int main() {
    long long* d; double* s;
    (void)hipMalloc(&d, 64); (void)hipMalloc(&s, 64 * 8);
    const int n = 2000;
    hipLaunchKernelGGL(lat, dim3(1), dim3(64), 0, 0, d, s, n);
    (void)hipDeviceSynchronize();
    hipLaunchKernelGGL(lat, dim3(1), dim3(64), 0, 0, d, s, n);
    long long h[5];
    (void)hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
    const double links = 8.0 * n;
    printf("fma f64 chain            %6.1f cycles/link\n", h[0] / links);
    printf("readlane x2 -> fma chain %6.1f cycles/link\n", h[1] / links);
    printf("ds_write/read -> fma     %6.1f cycles/link\n", h[2] / links);
    printf("mul f64 chain            %6.1f cycles/link\n", h[3] / links);
    printf("add + rcp f64 chain      %6.1f cycles/link\n", h[4] / links);
    return 0;
}
