// plant.hip — the bicycle plant around the SCP solve, batched on MI355X (fp64).
//
//   scpqp_delay_compensate  IterClass delay compensation: every vehicle of every
//                           problem integrated over delay_x + dt + delay_u with
//                           its last commanded steering (MPC_Iter.py:24-33)
//   scpqp_plant_step        closed-loop plant simulation over one MPC step
//                           (main.py:176-191)
//   scpqp_clip_controls     steering-limit enforcement of the controller output
//                           (main.py:164-174)
//
// The reference integrates with scipy (odeint = LSODA at rtol = atol = 1.49e-8
// for the delay compensation, dopri5 at rtol = atol = 1e-8 for the plant).
// Here every trajectory is one lane running the classical fourth-order
// Runge-Kutta method with a fixed step (default 2.5 ms, a quarter tick): the
// right-hand side is smooth, so the fixed step is ~1e-11 from the exact flow —
// three orders below the reference's own integration tolerance — and the
// lanes of a wave stay in lockstep (no adaptive step control to diverge on).
// The integration is compute-bound and tiny next to the SCP solve; the lanes
// read and write their 6-state rows directly (48 B per lane).
#include <hip/hip_runtime.h>

#include <math.h>

#include "scpqp.h"

int scpqp_fail_(int code, const char* msg);   // scpqp.hip: sets scpqp_last_error()

namespace {

constexpr int NX = 6;
constexpr int PT = 256;   // threads per workgroup

struct Veh {
    double lf, lr, uref, n0, n1;
};

// Model.py:61-87 (BicyleModel.ode / odes_): dx for state
// [x, y, heading, speed (rear axle), acceleration, steering angle].
// n0, n1: the additive noise of dx[0], dx[1] (Model.py:84-86), held constant
// over the call (the reference draws it anew per right-hand-side evaluation,
// and is_noise is False in main.py:235).
__device__ __forceinline__ void bicycle(const double (&x)[NX], const Veh& p, double (&dx)[NX]) {
    const double L = p.lf + p.lr, R = p.lr / L;
    const double tu = tan(x[5]);
    const double vc = x[3] * sqrt(1.0 + (R * tu) * (R * tu));
    const double beta = atan(R * tu);
    dx[0] = vc * cos(x[2] + beta) + p.n0;
    dx[1] = vc * sin(x[2] + beta) + p.n1;
    dx[2] = vc * tu * cos(beta) / L;
    dx[3] = x[4];
    dx[4] = 0.0;
    dx[5] = (p.uref - x[5]) / 0.1;
}

__device__ __forceinline__ void rk4(double (&x)[NX], const Veh& p, double h) {
    double k1[NX], k2[NX], k3[NX], k4[NX], y[NX];
    bicycle(x, p, k1);
#pragma unroll
    for (int i = 0; i < NX; ++i) y[i] = x[i] + 0.5 * h * k1[i];
    bicycle(y, p, k2);
#pragma unroll
    for (int i = 0; i < NX; ++i) y[i] = x[i] + 0.5 * h * k2[i];
    bicycle(y, p, k3);
#pragma unroll
    for (int i = 0; i < NX; ++i) y[i] = x[i] + h * k3[i];
    bicycle(y, p, k4);
#pragma unroll
    for (int i = 0; i < NX; ++i) x[i] += h / 6.0 * (k1[i] + 2.0 * k2[i] + 2.0 * k3[i] + k4[i]);
}

// integrate x over a span of length T with n equal RK4 steps
__device__ __forceinline__ void flow(double (&x)[NX], const Veh& p, double T, int n) {
    const double h = T / n;
    for (int s = 0; s < n; ++s) rk4(x, p, h);
}

__device__ __forceinline__ int steps_for(double T, double hmax) {
    const int n = (int)ceil(fabs(T) / hmax - 1e-9);
    return n < 1 ? 1 : n;
}

// one lane per (problem, vehicle): linspace(0, horizon, n_out) outputs
__global__ __launch_bounds__(PT) void delay_kernel(scpqp_plant_params p, int B, double horizon,
                                                   int n_out, double hmax, const double* x_meas,
                                                   const double* u_hold, const double* noise,
                                                   double* x0_out, double* traj_out) {
    const int V = p.n_veh;
    const int g = blockIdx.x * PT + threadIdx.x;
    if (g >= B * V) return;
    const int b = g / V, v = g % V;
    Veh q{p.lf[v], p.lr[v], u_hold[g], noise ? noise[2 * g] : 0.0, noise ? noise[2 * g + 1] : 0.0};
    double x[NX];
#pragma unroll
    for (int i = 0; i < NX; ++i) x[i] = x_meas[(size_t)g * NX + i];
    const double span = horizon / (n_out - 1);
    const int n = steps_for(span, hmax);
    for (int j = 0; j < n_out; ++j) {
        if (j > 0) flow(x, q, span, n);
        if (traj_out) {
            // MPC_delay_compensation_trajectory layout [n_out][nx][nVeh] per problem
#pragma unroll
            for (int i = 0; i < NX; ++i)
                traj_out[(((size_t)b * n_out + j) * NX + i) * V + v] = x[i];
        }
    }
#pragma unroll
    for (int i = 0; i < NX; ++i) x0_out[(size_t)g * NX + i] = x[i];
}

// one lane per (problem, vehicle, output tick k): main.py:186-190 restarts the
// integration at t0 for every output time t_k, with the control value of tick k
__global__ __launch_bounds__(PT) void plant_kernel(scpqp_plant_params p, int B, int n_ticks,
                                                   double tick, double hmax, const double* x_start,
                                                   const double* u_tick, const double* noise,
                                                   double* x_path) {
    const int V = p.n_veh, K = n_ticks + 1;
    const int g = blockIdx.x * PT + threadIdx.x;
    if (g >= B * V * K) return;
    const int k = g % K, bv = g / K, v = bv % V;
    Veh q{p.lf[v], p.lr[v], u_tick[g], noise ? noise[2 * bv] : 0.0,
          noise ? noise[2 * bv + 1] : 0.0};
    double x[NX];
#pragma unroll
    for (int i = 0; i < NX; ++i) x[i] = x_start[(size_t)bv * NX + i];
    if (k > 0) {
        const double T = k * tick;
        flow(x, q, T, steps_for(T, hmax));
    }
#pragma unroll
    for (int i = 0; i < NX; ++i) x_path[(size_t)g * NX + i] = x[i];
}

// one lane per (problem, vehicle): U[0] within +-umax and u0 +- du_lim, then
// U[j] within +-umax and U[j-1] +- du_lim (main.py:164-174), in place on the
// solver's vehicle-major layout u[v * hp + j]
__global__ __launch_bounds__(PT) void clip_kernel(int B, int V, int hp, int ld, double du_lim,
                                                  double* u, const double* u0, const double* umax) {
    const int g = blockIdx.x * PT + threadIdx.x;
    if (g >= B * V) return;
    const int b = g / V, v = g % V;
    double* uv = u + (size_t)b * ld + (size_t)v * hp;
    const double um = umax[g];
    double prev = u0[g];
    for (int j = 0; j < hp; ++j) {
        double w = uv[j];
        w = fmin(w, um);
        w = fmax(w, -um);
        w = fmin(w, prev + du_lim);
        w = fmax(w, prev - du_lim);
        uv[j] = w;
        prev = w;
    }
}

int check_params(const scpqp_plant_params* p) {
    if (!p) return scpqp_fail_(SCPQP_E_ARG, "null plant params");
    if (p->n_veh < 1 || p->n_veh > SCPQP_MAX_VEH) return scpqp_fail_(SCPQP_E_ARG, "n_veh out of range");
    for (int v = 0; v < p->n_veh; ++v)
        if (!(p->lf[v] + p->lr[v] > 0.0)) return scpqp_fail_(SCPQP_E_ARG, "lf + lr must be > 0");
    return 0;
}

int launched() {
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return scpqp_fail_(SCPQP_E_HIP, hipGetErrorString(e));
    return 0;
}

}  // namespace

extern "C" {

int scpqp_delay_compensate(const scpqp_plant_params* p, int32_t B, double horizon, int32_t n_out,
                           const double* x_meas, const double* u_hold, const double* noise,
                           double* x0_out, double* traj_out, double h_max, void* stream) {
    if (int rc = check_params(p)) return rc;
    if (B < 0) return scpqp_fail_(SCPQP_E_ARG, "batch size < 0");
    if (n_out < 2) return scpqp_fail_(SCPQP_E_ARG, "n_out must be >= 2");
    if (!(horizon >= 0.0) || !(h_max > 0.0)) return scpqp_fail_(SCPQP_E_ARG, "bad horizon / h_max");
    if (B == 0) return 0;
    if (!x_meas || !u_hold || !x0_out) return scpqp_fail_(SCPQP_E_ARG, "null array");
    const int n = B * p->n_veh;
    hipLaunchKernelGGL(delay_kernel, dim3((n + PT - 1) / PT), dim3(PT), 0,
                       static_cast<hipStream_t>(stream), *p, B, horizon, n_out, h_max, x_meas,
                       u_hold, noise, x0_out, traj_out);
    return launched();
}

int scpqp_plant_step(const scpqp_plant_params* p, int32_t B, int32_t n_ticks, double tick,
                     const double* x_start, const double* u_tick, const double* noise,
                     double* x_path, double h_max, void* stream) {
    if (int rc = check_params(p)) return rc;
    if (B < 0 || n_ticks < 0) return scpqp_fail_(SCPQP_E_ARG, "batch size / n_ticks < 0");
    if (!(tick > 0.0) || !(h_max > 0.0)) return scpqp_fail_(SCPQP_E_ARG, "bad tick / h_max");
    if (B == 0) return 0;
    if (!x_start || !u_tick || !x_path) return scpqp_fail_(SCPQP_E_ARG, "null array");
    const long long n = (long long)B * p->n_veh * (n_ticks + 1);
    if (n > 0x7fffffffLL) return scpqp_fail_(SCPQP_E_SIZE, "B * n_veh * (n_ticks + 1) too large");
    hipLaunchKernelGGL(plant_kernel, dim3((unsigned)((n + PT - 1) / PT)), dim3(PT), 0,
                       static_cast<hipStream_t>(stream), *p, B, n_ticks, tick, h_max, x_start,
                       u_tick, noise, x_path);
    return launched();
}

int scpqp_clip_controls(int32_t B, int32_t n_veh, int32_t hp, int32_t ld, double du_lim, double* u,
                        const double* u0, const double* umax, void* stream) {
    if (B < 0 || n_veh < 1 || hp < 1 || ld < n_veh * hp) return scpqp_fail_(SCPQP_E_ARG, "bad sizes");
    if (B == 0) return 0;
    if (!u || !u0 || !umax) return scpqp_fail_(SCPQP_E_ARG, "null array");
    const int n = B * n_veh;
    hipLaunchKernelGGL(clip_kernel, dim3((n + PT - 1) / PT), dim3(PT), 0,
                       static_cast<hipStream_t>(stream), B, n_veh, hp, ld, du_lim, u, u0, umax);
    return launched();
}

}  // extern "C"
