// Micro-benchmark: the row-by-row triangular solve (Solver) against the blocked solve
// with inverted 4 x 4 / 8 x 8 diagonal blocks (BSolver), n compile-time as in the c2
// kernel (81) and c5's Hp 30 (121).  One workgroup alone, 1 and 2 per CU.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include tools/probe/bsolve_probe.hip -o tools/probe/bsolve_probe
#include "../../senquential-convex-programming-for-trajectory-planning_amd/csrc/scpqp_kernel.h"

#include <vector>

// The blocked solve under test (not in the kernel: measured slower, DESIGN round 5).
namespace {
// ---------------------------------------------------------------------------
// Blocked solve with inverted diagonal blocks (LDS factors).  block_inverses()
// overwrites the strictly lower entries of every BS x BS diagonal block of the
// unit-lower L with those of X = L_kk^{-1} (blocks k = rows [BS k, BS k + BS)).  No
// later reader needs the L entries there: the panel steps read only rows below each
// panel's diagonal block, and the solves use X.  A solve then takes one v_readlane
// round per block instead of one per row: the block's BS right-hand sides are
// broadcast at once, the block's solution is X rb on uniform values (depth BS - 1
// FMAs), and every row takes the rank-BS update.  Per block of BS rows the chain is
// one readlane link, BS - 1 FMAs and one FMA of the update; the row-by-row sweep is
// BS readlane links.
// ---------------------------------------------------------------------------
constexpr int kSolveBlock = 4;

// X of every diagonal block, one lane per block (after the factorisation's last
// barrier); the caller synchronises before the solves.
template <int BS, class HP>
__device__ __forceinline__ void block_inverses(HP H, int n) {
    const int nblk = (n + BS - 1) / BS;
    for (int k = threadIdx.x; k < nblk; k += NT) {
        const int j0 = BS * k, bk = min(BS, n - j0);
        double l[BS][BS], x[BS][BS];
#pragma unroll
        for (int c = 1; c < BS; ++c)
#pragma unroll
            for (int m = 0; m < c; ++m) l[c][m] = c < bk ? (double)H[roff(j0 + c) + j0 + m] : 0.0;
        // X = L^{-1}, unit lower: X[c][m] = -L[c][m] - sum_{m < p < c} L[c][p] X[p][m]
#pragma unroll
        for (int c = 1; c < BS; ++c)
#pragma unroll
            for (int m = 0; m < c; ++m) {
                double s = -l[c][m];
#pragma unroll
                for (int p = m + 1; p < c; ++p) s = fma(-l[c][p], x[p][m], s);
                x[c][m] = s;
            }
#pragma unroll
        for (int c = 1; c < BS; ++c)
#pragma unroll
            for (int m = 0; m < c; ++m)
                if (c < bk) H[roff(j0 + c) + j0 + m] = x[c][m];
    }
}

// The lead wave only; rows i = lane + 64 t (t < R).  x: the solution (LDS); the block
// solutions are stored there by lane 0 as they are produced, so no lane captures its
// own entry.  The next block's X entries and L rows are loaded while the current block
// is solved (double buffer: the loads are issued before the block's stores to x, so
// their LDS latency is off the chain).
template <int R, int BS, class HP>
struct BSolver {
    static_assert(64 % BS == 0 && BS % 2 == 0, "blocks tile the 64-row slots");
    HP H;
    const ldouble* dinv;
    int lane, n;
    double r[R];
    int ro[R], ic[R];
    double xc[BS][BS], xn[BS][BS];   // X of the current / next block (strictly lower part)
    double lc[R][BS], ln[R][BS];     // L entries of the update, current / next block

    __device__ __forceinline__ BSolver(HP H_, const ldouble* dinv_, int n_, const ldouble* bvec)
        : H(H_), dinv(dinv_), n(n_) {
        lane = threadIdx.x & 63;
#pragma unroll
        for (int t = 0; t < R; ++t) {
            const int i = lane + 64 * t;
            ic[t] = i < n ? i : n - 1;
            ro[t] = roff(ic[t]);
            r[t] = i < n ? bvec[i] : 0.0;
        }
    }
    __device__ __forceinline__ void load_x(double (&X)[BS][BS], int j0) {
        const int bk = min(BS, n - j0);
#pragma unroll
        for (int c = 1; c < BS; ++c)
#pragma unroll
            for (int m = 0; m < c; ++m) X[c][m] = c < bk ? (double)H[roff(j0 + c) + j0 + m] : 0.0;
    }
    // forward: row entries L[i][j0 .. j0 + BS) of slots t >= T0
    template <int T0>
    __device__ __forceinline__ void load_fwd(double (&X)[BS][BS], double (&Lr)[R][BS], int j0) {
        load_x(X, j0);
#pragma unroll
        for (int t = T0; t < R; ++t)
#pragma unroll
            for (int c = 0; c < BS; c += 2) {
                const double2v v = ld2(H + ro[t] + j0 + c);
                Lr[t][c] = v.x;
                Lr[t][c + 1] = v.y;
            }
    }
    // backward: column entries L[j0 + c][i] of slots t <= T1
    template <int T1>
    __device__ __forceinline__ void load_bwd(double (&X)[BS][BS], double (&Lr)[R][BS], int j0) {
        load_x(X, j0);
        const int bk = min(BS, n - j0);
#pragma unroll
        for (int c = 0; c < BS; ++c) {
            const int row = c < bk ? j0 + c : j0;
#pragma unroll
            for (int t = 0; t <= T1 && t < R; ++t) Lr[t][c] = H[roff(row) + ic[t]];
        }
    }
    __device__ __forceinline__ void shift() {
#pragma unroll
        for (int c = 0; c < BS; ++c) {
#pragma unroll
            for (int m = 0; m < BS; ++m) xc[c][m] = xn[c][m];
#pragma unroll
            for (int t = 0; t < R; ++t) lc[t][c] = ln[t][c];
        }
    }
    // One block at a time: the updates of every slot are kept in their block (else they
    // sink towards their first reader, the next slot's sweep, and the loaded L entries
    // they need pile up and spill), and the scheduler does not hoist later blocks' loads.
    __device__ __forceinline__ void pin() {
#pragma unroll
        for (int t = 0; t < R; ++t) asm volatile("" : "+v"(r[t]));
        __builtin_amdgcn_sched_barrier(0);
    }
    // the block's solution (uniform) to x[j0 .. j0 + bk)
    __device__ __forceinline__ void put(ldouble* x, int j0, int bk, const double (&y)[BS]) {
        if (lane == 0) {
#pragma unroll
            for (int c = 0; c < BS; c += 2) {
                if (c + 1 < bk) st2(x + j0 + c, double2v{y[c], y[c + 1]});
                else if (c < bk) x[j0 + c] = y[c];
            }
        }
    }
    // forward L y = b over the blocks owned by slot T (rows 64 T .. 64 T + 63)
    template <int T>
    __device__ __forceinline__ void fwd(ldouble* x) {
        if constexpr (T < R) {
            const int jend = min(n, 64 * (T + 1));
            for (int j0 = 64 * T; j0 < jend; j0 += BS) {
                const int bk = min(BS, n - j0);
                if (j0 + BS < n) load_fwd<T>(xn, ln, j0 + BS);
                double rb[BS], y[BS];
#pragma unroll
                for (int c = 0; c < BS; ++c) rb[c] = c < bk ? readlane_d(r[T], (j0 + c) & 63) : 0.0;
                // y = X rb (X unit lower)
#pragma unroll
                for (int c = 0; c < BS; ++c) {
                    double s = rb[c];
#pragma unroll
                    for (int m = 0; m < c; ++m) s = fma(xc[c][m], rb[m], s);
                    y[c] = c < bk ? s : 0.0;
                }
                put(x, j0, bk, y);
                // rank-BS update of the rows below (rows at or above the block: garbage)
#pragma unroll
                for (int t = T; t < R; ++t)
#pragma unroll
                    for (int c = 0; c < BS; ++c)
                        if (c < bk) r[t] = fma(-lc[t][c], y[c], r[t]);
                shift();
                pin();
            }
        }
    }
    // backward L' x = z over the blocks owned by slot T, last block first
    template <int T>
    __device__ __forceinline__ void bwd(ldouble* x, int jlast) {
        if constexpr (T < R) {
            const int jstart = (T == R - 1) ? jlast : 64 * T + 64 - BS;
            for (int j0 = jstart; j0 >= 64 * T; j0 -= BS) {
                const int bk = min(BS, n - j0);
                if (j0 > 0) load_bwd<T>(xn, ln, j0 - BS);
                double rb[BS], y[BS];
#pragma unroll
                for (int c = 0; c < BS; ++c) rb[c] = c < bk ? readlane_d(r[T], (j0 + c) & 63) : 0.0;
                // y = X' rb
#pragma unroll
                for (int c = BS - 1; c >= 0; --c) {
                    double s = rb[c];
#pragma unroll
                    for (int m = BS - 1; m > c; --m)
                        if (m < bk) s = fma(xc[m][c], rb[m], s);
                    y[c] = c < bk ? s : 0.0;
                }
                put(x, j0, bk, y);
                // rows above the block: r_i -= sum_c L[j0 + c][i] y_c (the last entry first)
#pragma unroll
                for (int t = 0; t <= T; ++t)
#pragma unroll
                    for (int c = BS - 1; c >= 0; --c)
                        if (c < bk) r[t] = fma(-lc[t][c], y[c], r[t]);
                shift();
                pin();
            }
        }
    }
    __device__ __forceinline__ void run(ldouble* x) {
        PROF_T0();
        load_fwd<0>(xc, lc, 0);
        fwd<0>(x); fwd<1>(x); fwd<2>(x); fwd<3>(x);
        PROF_ACC(14);
        // z = D^{-1} y: each lane reads back its own entries (same wave: LDS in order)
#pragma unroll
        for (int t = 0; t < R; ++t) r[t] = x[ic[t]] * dinv[ic[t]];
        const int jlast = ((n - 1) / BS) * BS;
        load_bwd<R - 1>(xc, lc, jlast);
        bwd<3>(x, jlast); bwd<2>(x, jlast); bwd<1>(x, jlast); bwd<0>(x, jlast);
        PROF_ACC(15);
    }
};
}  // namespace


namespace {
// Rolled blocked solve (one runtime loop per 64-row slot, BS = 4): the next block's X
// entries and L entries are loaded one block ahead, every block's solution is captured
// into its owner lanes with v_cndmask (no store, no branch), and a partial last block
// is masked by zeroing its missing solution entries.
template <int R, int BS, class HP>
struct BSolver2 {
    HP H;
    const ldouble* dinv;
    int lane, n;
    double r[R], xf[R];
    int ro[R], ic[R];
    __device__ __forceinline__ BSolver2(HP H_, const ldouble* dinv_, int n_, const ldouble* bvec)
        : H(H_), dinv(dinv_), n(n_) {
        lane = threadIdx.x & 63;
#pragma unroll
        for (int t = 0; t < R; ++t) {
            const int i = lane + 64 * t;
            ic[t] = i < n ? i : n - 1;
            ro[t] = roff(ic[t]);
            r[t] = i < n ? bvec[i] : 0.0;
            xf[t] = 0.0;
        }
    }
    struct Blk {
        double x[BS * (BS - 1) / 2];
        double l[R][BS];
    };
    __device__ __forceinline__ void load_x(Blk& b, int j0) {
        int q = 0;
#pragma unroll
        for (int c = 1; c < BS; ++c)
#pragma unroll
            for (int m = 0; m < c; ++m) b.x[q++] = H[roff(j0 + c) + j0 + m];
    }
    template <int T0>
    __device__ __forceinline__ void load_f(Blk& b, int j0) {
        load_x(b, j0);
#pragma unroll
        for (int t = T0; t < R; ++t)
#pragma unroll
            for (int c = 0; c < BS; c += 2) {
                const double2v v = ld2(H + ro[t] + j0 + c);
                b.l[t][c] = v.x;
                b.l[t][c + 1] = v.y;
            }
    }
    template <int T1>
    __device__ __forceinline__ void load_b(Blk& b, int j0) {
        load_x(b, j0);
#pragma unroll
        for (int c = 0; c < BS; ++c) {
            const int row = min(j0 + c, n - 1);
#pragma unroll
            for (int t = 0; t <= T1 && t < R; ++t) b.l[t][c] = H[roff(row) + ic[t]];
        }
    }
    template <int T>
    __device__ __forceinline__ void fwd(Blk& cur) {
        if constexpr (T < R) {
            const int jend = min(n, 64 * (T + 1));
#pragma unroll 1
            for (int j0 = 64 * T; j0 < jend; j0 += BS) {
                Blk nxt;
                if (j0 + BS < n) load_f<T>(nxt, j0 + BS);
                double rb[BS], y[BS];
#pragma unroll
                for (int c = 0; c < BS; ++c) rb[c] = readlane_d(r[T], (j0 + c) & 63);
                int q = 0;
#pragma unroll
                for (int c = 0; c < BS; ++c) {
                    double s = rb[c];
#pragma unroll
                    for (int m = 0; m < c; ++m) s = fma(cur.x[q++], rb[m], s);
                    y[c] = j0 + c < n ? s : 0.0;
                    xf[T] = lane == ((j0 + c) & 63) ? y[c] : xf[T];
                }
#pragma unroll
                for (int t = T; t < R; ++t)
#pragma unroll
                    for (int c = 0; c < BS; ++c) r[t] = fma(-cur.l[t][c], y[c], r[t]);
                cur = nxt;
            }
        }
    }
    template <int T>
    __device__ __forceinline__ void bwd(Blk& cur, int jlast) {
        if constexpr (T < R) {
            const int jstart = (T == R - 1) ? jlast : 64 * T + 64 - BS;
#pragma unroll 1
            for (int j0 = jstart; j0 >= 64 * T; j0 -= BS) {
                Blk nxt;
                if (j0 > 0) load_b<T>(nxt, j0 - BS);
                double rb[BS], y[BS];
#pragma unroll
                for (int c = 0; c < BS; ++c) rb[c] = readlane_d(r[T], (j0 + c) & 63);
#pragma unroll
                for (int c = BS - 1; c >= 0; --c) {
                    double s = rb[c];
#pragma unroll
                    for (int m = BS - 1; m > c; --m) {
                        const int q = m * (m - 1) / 2 + c;   // X[m][c]
                        s = fma(cur.x[q], j0 + m < n ? rb[m] : 0.0, s);
                    }
                    y[c] = j0 + c < n ? s : 0.0;
                    xf[T] = lane == ((j0 + c) & 63) ? y[c] : xf[T];
                }
#pragma unroll
                for (int t = 0; t <= T; ++t)
#pragma unroll
                    for (int c = BS - 1; c >= 0; --c) r[t] = fma(-cur.l[t][c], y[c], r[t]);
                cur = nxt;
            }
        }
    }
    __device__ __forceinline__ void run(ldouble* x) {
        Blk cur;
        load_f<0>(cur, 0);
        fwd<0>(cur); fwd<1>(cur); fwd<2>(cur); fwd<3>(cur);
#pragma unroll
        for (int t = 0; t < R; ++t) {
            r[t] = xf[t] * dinv[ic[t]];
            xf[t] = 0.0;
        }
        const int jlast = ((n - 1) / BS) * BS;
        load_b<R - 1>(cur, jlast);
        bwd<3>(cur, jlast); bwd<2>(cur, jlast); bwd<1>(cur, jlast); bwd<0>(cur, jlast);
#pragma unroll
        for (int t = 0; t < R; ++t)
            if (lane + 64 * t < n) x[lane + 64 * t] = xf[t];
    }
};
}  // namespace

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
    if (VAR == 1 || VAR == 3) block_inverses<4>(H, n);
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
            } else if constexpr (VAR == 2) {
                BSolver<R, 8, ldouble*> S(H, dinv, n, b);
                S.run(x);
            } else {
                BSolver2<R, 4, ldouble*> S(H, dinv, n, b);
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
        run<3, NC>("BSolver2<4>", grid, 50, dx, dc, xr.data());
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
