// c3 factor on chip (verdict r05 item 4, SURVEY §7 option (a)): a probe of the
// L D L' factorisation of c3's 241 x 241 normal matrix with the whole factor on one
// CU, against the shipped kernel's factorisation (plan 2: packed factor in the
// global workspace, two workgroups per CU, lead-wave panels of 8 + grouped MFMA
// trailing update).  Factorisation only: no assembly, no solves.
//
// On-chip layout (one 256-thread workgroup per CU): n padded to 256 = 16 tile rows
// of 16 (rows 241..255 an identity block), 136 lower tiles of 16 x 16 f64.  The 4 RT
// most-updated tiles (highest tile column first) live in the waves' registers as
// v_mfma_f64_16x16x4_f64 accumulators (RT per wave, compile-time indexed); the rest
// in LDS, column-major with a column stride of 17 (conflict-free both for the MFMA
// operand reads, rows along lanes, and for the accumulator reads, columns along
// lanes).  Right-looking by tile column k:
//   (a) register tiles of column k -> the LDS panel buffer P;
//   (b) wave 0 factors the diagonal tile (16 pivots, v_readlane broadcasts);
//   (c) every thread solves one panel row against it (forward substitution);
//   (d) every wave updates its tiles right of k with 4 MFMAs each (rank 16), operands
//       read from the panel in LDS, and takes its register tiles of column k back.
// Four barriers per tile column, 16 columns.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include tools/probe/c3_onchip_probe.hip \
//         -o tools/probe/c3_onchip_probe
// Output: cycles (s_memtime) per factorisation, alone and with every CU busy, and
// the factorisations per second of the whole chip (kernel wall time), for both.
#include "../../senquential-convex-programming-for-trajectory-planning_amd/csrc/scpqp_kernel.h"
#include <algorithm>
#include <cmath>
#include <vector>

namespace {
constexpr int NN = 241;          // c3: 8 vehicles x Hp 30 + the slack
constexpr int TN = 16;           // tile rows (n padded to 256)
constexpr int CS = 17;           // column stride of an LDS tile
constexpr int TS = 16 * CS;      // doubles per LDS tile (272)
constexpr int NTILE = TN * (TN + 1) / 2;


// tiles in the order (tile column J descending, tile row I descending): index t -> (I, J).
// The first 4 RT are register tiles (wave t % 4, slot t / 4; P slot 15 - I), the rest LDS
// tiles (slot t - 4 RT, wave (t - 4 RT) % 4).  Decoded arithmetically inside the loop:
// a table of 3 RT uniform values per wave, hoisted, spills the scalar file.
__host__ __device__ __forceinline__ void tdecode(int t, int& I, int& J) {
    int m = (int)((sqrtf(8.0f * t + 1.0f) - 1.0f) * 0.5f);
    if ((m + 1) * (m + 2) / 2 <= t) ++m;
    if (m * (m + 1) / 2 > t) --m;
    J = TN - 1 - m;
    I = TN - 1 - (t - m * (m + 1) / 2);
}
__host__ __device__ __forceinline__ int tindex(int I, int J) {
    return (TN - 1 - J) * (TN - J) / 2 + (TN - 1 - I);
}
// per-wave slot tables and the panel-operand offsets, read with scalar loads inside the
// column loop (indexed through an opaque copy of the wave id so that they are not
// hoisted: hoisted they spill the scalar file)
__constant__ int c_slot[4][32];    // I | J << 8 of register slot s (-1: none)
__constant__ int c_base[TN][TN];   // LDS offset of tile (I, J) as a panel operand
// an opaque copy: values derived from it are recomputed where they are used
__device__ __forceinline__ int opaque(int v) {
    asm volatile("" : "+s"(v));
    return v;
}

__device__ __forceinline__ double kval(const double* K, int i, int j) {
    if (i < NN && j < NN) return K[i * NN + j];
    return i == j ? 1.0 : 0.0;
}

template <int RT>
__global__ __launch_bounds__(256, 1) void onchip_factor(const double* K, double* Lout, long long* cyc, int reps,
                                                         int pbase, int dbase) {
    constexpr int NREG = 4 * RT < NTILE ? 4 * RT : NTILE;
    constexpr int NLDS = NTILE - NREG;
    ldouble* S = (ldouble*)smem_;
    const int lane = threadIdx.x & 63, w0 = wave_id();
    const int lr = lane & 15, lk = lane >> 4;
    double4v acc[RT];
    long long tot = 0, ph[4] = {0, 0, 0, 0};
    for (int rep = 0; rep < reps; ++rep) {
        // the matrix (untimed): register tiles in C/D layout, LDS tiles column-major
#pragma unroll
        for (int s = 0; s < RT; ++s) {
            const int t = 4 * s + w0;
            int I = 0, J = 0;
            tdecode(t, I, J);
#pragma unroll
            for (int r = 0; r < 4; ++r) acc[s][r] = t < NREG ? kval(K, 16 * I + lk + 4 * r, 16 * J + lr) : 0.0;
        }
        for (int t = NREG + w0; t < NTILE; t += 4) {
            int I, J;
            tdecode(t, I, J);
            ldouble* T = S + (t - NREG) * TS;
#pragma unroll
            for (int r = 0; r < 4; ++r) T[lr * CS + lk + 4 * r] = kval(K, 16 * I + lk + 4 * r, 16 * J + lr);
        }
        __syncthreads();
        const long long t0 = __builtin_amdgcn_s_memtime();
        ldouble* Dd = S + dbase;
        ldouble* Di = Dd + 16;
        for (int k = 0; k < TN; ++k) {
            const int w = opaque(w0);
            // (a) register tiles of column k into P: slots with tk <= 4 s + w < tk + 16 - k
            const int tk = tindex(TN - 1, k);   // first tile of column k (row 15)
#pragma unroll
            for (int s = 0; s < RT; ++s) {
                const int t = 4 * s + w;
                if (t < NREG && t >= tk && t < tk + TN - k) {
                    ldouble* T = S + pbase + (t - tk) * TS;   // P slot 15 - I
#pragma unroll
                    for (int r = 0; r < 4; ++r) T[lr * CS + lk + 4 * r] = acc[s][r];
                }
            }
            __syncthreads();
            long long tp = __builtin_amdgcn_s_memtime();
            ph[0] += tp;
            // (b) the diagonal tile, wave 0: lane r (< 16) holds row r
            ldouble* B0 = S + c_base[k][k];
            if (w == 0) {
                // symmetric elimination: row c of the updated tile (lane c, the tile is kept
                // symmetric by the full-tile MFMA updates) is broadcast before the pivot's
                // reciprocal is formed, so the chain per pivot is one v_readlane round
                double a[16];
#pragma unroll
                for (int c = 0; c < 16; ++c) a[c] = B0[c * CS + lr];
#pragma unroll
                for (int c = 0; c < 16; ++c) {
                    double rc[16];
#pragma unroll
                    for (int c2 = c; c2 < 16; ++c2) rc[c2] = readlane_d(a[c2], c);
                    const double d = rc[c];
                    const double ri = recip(d);
                    const double l = a[c] * ri;
#pragma unroll
                    for (int c2 = c + 1; c2 < 16; ++c2) a[c2] = fma(-l, rc[c2], a[c2]);
                    a[c] = lr > c ? l : (lr == c ? d : 0.0);
                    if (lane == c) {
                        Dd[c] = d;
                        Di[c] = ri;
                    }
                }
                if (lane < 16) {
#pragma unroll
                    for (int c = 0; c < 16; ++c) B0[c * CS + lr] = a[c];
                }
            }
            __syncthreads();
            {
                const long long t2 = __builtin_amdgcn_s_memtime();
                ph[1] += t2 - tp;
                tp = t2;
            }
            // (c) panel rows below the diagonal tile: y = a - sum y_c' L_kk[c][c'], l = y / d
            {
                const int rho = 16 * (k + 1) + (int)threadIdx.x;
                if (rho < 16 * TN) {
                    ldouble* Bi = S + c_base[rho >> 4][k];
                    const int row = rho & 15;
                    // right-looking: y_c' leaves the chain as soon as it is final
                    double y[16];
#pragma unroll
                    for (int c = 0; c < 16; ++c) y[c] = Bi[c * CS + row];
#pragma unroll
                    for (int c2 = 0; c2 < 15; ++c2) {
                        double lc[16];
#pragma unroll
                        for (int c = c2 + 1; c < 16; ++c) lc[c] = B0[c2 * CS + c];
#pragma unroll
                        for (int c = c2 + 1; c < 16; ++c) y[c] = fma(-y[c2], lc[c], y[c]);
                    }
#pragma unroll
                    for (int c = 0; c < 16; ++c) Bi[c * CS + row] = y[c] * Di[c];
                }
            }
            __syncthreads();
            {
                const long long t2 = __builtin_amdgcn_s_memtime();
                ph[2] += t2 - tp;
                tp = t2;
            }
            // (d) register tiles of column k back; trailing update of tiles right of k
            const int w2 = opaque(w0);
            double dq[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) dq[q] = -Dd[4 * q + lk];
            // register tiles right of k: the slots 4 s + w2 < tk, a prefix (slot tile columns
            // descend); in groups of four whose MFMA chains interleave (an idle slot of the
            // last group gets a zero A operand and reads the diagonal tile's panel rows)
            const int nact = (tk - w2 + 3) >> 2;
#pragma unroll
            for (int g = 0; g < RT; g += 4) {
                if (g < nact) {
                    double av[4][4], bv[4][4];
                    const int* slot = c_slot[w2];
#pragma unroll
                    for (int u = 0; u < 4; ++u) {
                        const bool act = g + u < nact && g + u < RT;
                        const int ij = act ? slot[g + u] : (k | (k << 8));
                        const ldouble* A = S + c_base[ij & 255][k];
                        const ldouble* Bt = S + c_base[ij >> 8][k];
#pragma unroll
                        for (int q = 0; q < 4; ++q) {
                            av[u][q] = A[(4 * q + lk) * CS + lr] * (act ? dq[q] : 0.0);
                            bv[u][q] = Bt[(4 * q + lk) * CS + lr];
                        }
                    }
#pragma unroll
                    for (int q = 0; q < 4; ++q)
#pragma unroll
                        for (int u = 0; u < 4; ++u)
                            if (g + u < RT)
                                acc[g + u] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[u][q], bv[u][q], acc[g + u], 0, 0, 0);
                }
            }
            // register tiles of column k back from P
#pragma unroll
            for (int s = 0; s < RT; ++s) {
                const int t = 4 * s + w2;
                if (t < NREG && t >= tk && t < tk + TN - k) {
                    const ldouble* T = S + pbase + (t - tk) * TS;
#pragma unroll
                    for (int r = 0; r < 4; ++r) acc[s][r] = T[lr * CS + lk + 4 * r];
                }
            }
            // LDS tiles right of k: the indices below the first tile of column k
            for (int t = NREG + w2; t < tk; t += 4) {
                int I, J;
                tdecode(t, I, J);
                const ldouble* A = S + c_base[I][k];
                const ldouble* Bt = S + c_base[J][k];
                ldouble* T = S + (t - NREG) * TS;
                double av[4], bv[4];
                double4v c4;
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    av[q] = A[(4 * q + lk) * CS + lr] * dq[q];
                    bv[q] = Bt[(4 * q + lk) * CS + lr];
                }
#pragma unroll
                for (int r = 0; r < 4; ++r) c4[r] = T[lr * CS + lk + 4 * r];
#pragma unroll
                for (int q = 0; q < 4; ++q) c4 = __builtin_amdgcn_mfma_f64_16x16x4f64(av[q], bv[q], c4, 0, 0, 0);
#pragma unroll
                for (int r = 0; r < 4; ++r) T[lr * CS + lk + 4 * r] = c4[r];
            }
            __syncthreads();
            {
                const long long t2 = __builtin_amdgcn_s_memtime();
                ph[3] += t2 - tp;
                ph[0] -= t2;   // (a): from here to the first barrier of the next column
            }
        }
        ph[0] += __builtin_amdgcn_s_memtime();
        tot += __builtin_amdgcn_s_memtime() - t0;
    }
    if (threadIdx.x == 0) cyc[blockIdx.x] = tot;
    if (threadIdx.x == 0 && blockIdx.x == 0)
        for (int i = 0; i < 4; ++i) cyc[4096 + i] = ph[i];
    if (blockIdx.x == 0) {
        // the factor (unit-lower L below the diagonal, D on it), dense 256 x 256
#pragma unroll
        for (int s = 0; s < RT; ++s) {
            const int t = 4 * s + w0;
            int I, J;
            tdecode(t, I, J);
            if (t < NREG) {
#pragma unroll
                for (int r = 0; r < 4; ++r) Lout[(16 * I + lk + 4 * r) * 256 + 16 * J + lr] = acc[s][r];
            }
        }
        for (int t = NREG + w0; t < NTILE; t += 4) {
            int I, J;
            tdecode(t, I, J);
            const ldouble* T = S + (t - NREG) * TS;
#pragma unroll
            for (int r = 0; r < 4; ++r) Lout[(16 * I + lk + 4 * r) * 256 + 16 * J + lr] = T[lr * CS + lk + 4 * r];
        }
    }
    (void)NLDS;
}

// ---------------------------------------------------------------------------
// Look-ahead variant: wave 0 is the panel wave (diagonal tile + panel rows, no tiles of
// its own), waves 1..3 hold the tiles (3 RT register tiles, the rest in LDS) and run the
// trailing update.  Step k: the tile waves update column k + 1 first and hand it over
// (P[(k + 1) & 1]); after one barrier wave 0 factors panel k + 1 while the tile waves
// apply panel k to the columns right of k + 1; a second barrier ends the step.  The
// panel buffer P and the pivots are double-buffered by column parity.
__constant__ int c_slot3[4][32];     // waves 1..3: I | J << 8 of register slot s
__constant__ int c_base3[TN][TN];    // LDS offset of tile (I, J) (P[J & 1] for register tiles)

// wave 0: L D L' of the diagonal tile at B0 (symmetric elimination, as above)
__device__ __forceinline__ void la_diag(ldouble* B0, ldouble* Dd, ldouble* Di, int lane) {
    const int lr = lane & 15;
    double a[16];
#pragma unroll
    for (int c = 0; c < 16; ++c) a[c] = B0[c * CS + lr];
#pragma unroll
    for (int c = 0; c < 16; ++c) {
        double rc[16];
#pragma unroll
        for (int c2 = c; c2 < 16; ++c2) rc[c2] = readlane_d(a[c2], c);
        const double d = rc[c];
        const double ri = recip(d);
        const double l = a[c] * ri;
#pragma unroll
        for (int c2 = c + 1; c2 < 16; ++c2) a[c2] = fma(-l, rc[c2], a[c2]);
        a[c] = lr > c ? l : (lr == c ? d : 0.0);
        if (lane == c) {
            Dd[c] = d;
            Di[c] = ri;
        }
    }
    if (lane < 16) {
#pragma unroll
        for (int c = 0; c < 16; ++c) B0[c * CS + lr] = a[c];
    }
}

// wave 0: the panel rows below the diagonal tile of column m, two rows per lane per pass
__device__ __forceinline__ void la_rows(ldouble* S, int m, const ldouble* B0, const ldouble* Di, int lane) {
    constexpr int RW = 2;
    for (int p0 = 16 * (m + 1); p0 < 16 * TN; p0 += 64 * RW) {
        ldouble* Bi[RW];
        int row[RW];
        bool ok[RW];
        double y[RW][16];
#pragma unroll
        for (int i = 0; i < RW; ++i) {
            const int rho = p0 + lane + 64 * i;
            ok[i] = rho < 16 * TN;
            Bi[i] = S + c_base3[ok[i] ? rho >> 4 : m][m];
            row[i] = rho & 15;
#pragma unroll
            for (int c = 0; c < 16; ++c) y[i][c] = Bi[i][c * CS + row[i]];
        }
#pragma unroll
        for (int c2 = 0; c2 < 15; ++c2) {
            double lc[16];
#pragma unroll
            for (int c = c2 + 1; c < 16; ++c) lc[c] = B0[c2 * CS + c];
#pragma unroll
            for (int i = 0; i < RW; ++i)
#pragma unroll
                for (int c = c2 + 1; c < 16; ++c) y[i][c] = fma(-y[i][c2], lc[c], y[i][c]);
        }
#pragma unroll
        for (int i = 0; i < RW; ++i)
            if (ok[i]) {
#pragma unroll
                for (int c = 0; c < 16; ++c) Bi[i][c * CS + row[i]] = y[i][c] * Di[c];
            }
    }
}

// tile waves: the register slots [slo, shi) (their tiles right of column k) receive panel k,
// four MFMA chains interleaved
template <int RT>
__device__ __forceinline__ void la_update_reg(double4v (&acc)[RT], const int* slot, int slo, int shi, int k,
                                              const ldouble* S, const double (&dq)[4], int lr, int lk) {
#pragma unroll
    for (int g = 0; g < RT; g += 4) {
        if (g + 3 >= slo && g < shi) {
            double av[4][4], bv[4][4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const bool act = g + u >= slo && g + u < shi && g + u < RT;
                const int ij = act ? slot[g + u] : (k | (k << 8));
                const ldouble* A = S + c_base3[ij & 255][k];
                const ldouble* Bt = S + c_base3[ij >> 8][k];
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    av[u][q] = A[(4 * q + lk) * CS + lr] * (act ? dq[q] : 0.0);
                    bv[u][q] = Bt[(4 * q + lk) * CS + lr];
                }
            }
#pragma unroll
            for (int q = 0; q < 4; ++q)
#pragma unroll
                for (int u = 0; u < 4; ++u)
                    if (g + u < RT)
                        acc[g + u] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[u][q], bv[u][q], acc[g + u], 0, 0, 0);
        }
    }
}

// tile waves: LDS tiles t in [tlo, thi) of this wave (t = NREG + 3 q + w - 1) receive panel k
__device__ __forceinline__ void la_update_lds(ldouble* S, int nreg, int tlo, int thi, int w, int k,
                                              const double (&dq)[4], int lr, int lk) {
    int t = nreg + w - 1;
    if (t < tlo) t += ((tlo - t + 2) / 3) * 3;
    for (; t < thi; t += 3) {
        int I, J;
        tdecode(t, I, J);
        const ldouble* A = S + c_base3[I][k];
        const ldouble* Bt = S + c_base3[J][k];
        ldouble* T = S + (t - nreg) * TS;
        double av[4], bv[4];
        double4v c4;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            av[q] = A[(4 * q + lk) * CS + lr] * dq[q];
            bv[q] = Bt[(4 * q + lk) * CS + lr];
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) c4[r] = T[lr * CS + lk + 4 * r];
#pragma unroll
        for (int q = 0; q < 4; ++q) c4 = __builtin_amdgcn_mfma_f64_16x16x4f64(av[q], bv[q], c4, 0, 0, 0);
#pragma unroll
        for (int r = 0; r < 4; ++r) T[lr * CS + lk + 4 * r] = c4[r];
    }
}

template <int RT>
__global__ __launch_bounds__(256, 1) void onchip_factor_la(const double* K, double* Lout, long long* cyc, int reps,
                                                            int pb0, int pb1, int dbase) {
    constexpr int NREG = 3 * RT < NTILE ? 3 * RT : NTILE;
    ldouble* S = (ldouble*)smem_;
    const int lane = threadIdx.x & 63, w0 = wave_id();
    const int lr = lane & 15, lk = lane >> 4;
    double4v acc[RT];
    long long tot = 0, ph[4] = {0, 0, 0, 0};
    // register slot s of wave w >= 1 holds tile t = 3 s + w - 1; slot range of tiles [ta, tb)
    auto srange = [&](int w, int ta, int tb, int& slo, int& shi) {
        slo = ta - (w - 1) <= 0 ? 0 : (ta - (w - 1) + 2) / 3;
        shi = tb - (w - 1) <= 0 ? 0 : (tb - (w - 1) + 2) / 3;
        if (shi > RT) shi = RT;
    };
    for (int rep = 0; rep < reps; ++rep) {
        if (w0 > 0) {
#pragma unroll
            for (int s = 0; s < RT; ++s) {
                const int t = 3 * s + w0 - 1;
                int I = 0, J = 0;
                tdecode(t < NREG ? t : 0, I, J);
#pragma unroll
                for (int r = 0; r < 4; ++r) acc[s][r] = t < NREG ? kval(K, 16 * I + lk + 4 * r, 16 * J + lr) : 0.0;
            }
            for (int t = NREG + w0 - 1; t < NTILE; t += 3) {
                int I, J;
                tdecode(t, I, J);
                ldouble* T = S + (t - NREG) * TS;
#pragma unroll
                for (int r = 0; r < 4; ++r) T[lr * CS + lk + 4 * r] = kval(K, 16 * I + lk + 4 * r, 16 * J + lr);
            }
        }
        __syncthreads();
        const long long t0 = __builtin_amdgcn_s_memtime();
        // prologue: column 0's register tiles to P[0]; wave 0 factors panel 0
        if (w0 > 0) {
            const int w = opaque(w0);
            int slo, shi;
            srange(w, 0, TN, slo, shi);
#pragma unroll
            for (int s = 0; s < RT; ++s) {
                const int t = 3 * s + w - 1;
                if (s >= slo && s < shi && t < NREG) {
                    ldouble* T = S + pb0 + t * TS;
#pragma unroll
                    for (int r = 0; r < 4; ++r) T[lr * CS + lk + 4 * r] = acc[s][r];
                }
            }
        }
        __syncthreads();
        if (w0 == 0) {
            ldouble* B0 = S + c_base3[0][0];
            la_diag(B0, S + dbase, S + dbase + 16, lane);
            la_rows(S, 0, B0, S + dbase + 16, lane);
        }
        __syncthreads();
        for (int k = 0; k < TN; ++k) {
            const long long ts = __builtin_amdgcn_s_memtime();
            const int w = opaque(w0);
            const int tk = tindex(TN - 1, k), tk1 = k + 1 < TN ? tindex(TN - 1, k + 1) : 0;
            ldouble* Dk = S + dbase + 32 * (k & 1);
            double dq[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) dq[q] = -Dk[4 * q + lk];
            if (w > 0) {
                const int* slot = c_slot3[w];
                const int pk = (k & 1) ? pb1 : pb0, pk1 = (k & 1) ? pb0 : pb1;
                int slo, shi;
                // column k's register tiles back (panel k is final)
                srange(w, tk, tk + TN - k, slo, shi);
#pragma unroll
                for (int s = 0; s < RT; ++s) {
                    const int t = 3 * s + w - 1;
                    if (s >= slo && s < shi && t < NREG) {
                        const ldouble* T = S + pk + (t - tk) * TS;
#pragma unroll
                        for (int r = 0; r < 4; ++r) acc[s][r] = T[lr * CS + lk + 4 * r];
                    }
                }
                if (k + 1 < TN) {
                    // column k + 1 first, then handed over to wave 0
                    srange(w, tk1, tk, slo, shi);
                    la_update_reg<RT>(acc, slot, slo, shi, k, S, dq, lr, lk);
                    la_update_lds(S, NREG, tk1 > NREG ? tk1 : NREG, tk, w, k, dq, lr, lk);
#pragma unroll
                    for (int s = 0; s < RT; ++s) {
                        const int t = 3 * s + w - 1;
                        if (s >= slo && s < shi && t < NREG) {
                            ldouble* T = S + pk1 + (t - tk1) * TS;
#pragma unroll
                            for (int r = 0; r < 4; ++r) T[lr * CS + lk + 4 * r] = acc[s][r];
                        }
                    }
                }
            }
            __syncthreads();
            const long long tb1 = __builtin_amdgcn_s_memtime();
            if (w == 0) {
                if (k + 1 < TN) {
                    ldouble* Dn = S + dbase + 32 * ((k + 1) & 1);
                    ldouble* B0 = S + c_base3[k + 1][k + 1];
                    la_diag(B0, Dn, Dn + 16, lane);
                    la_rows(S, k + 1, B0, Dn + 16, lane);
                }
                ph[2] += __builtin_amdgcn_s_memtime() - tb1;
            } else if (k + 1 < TN) {
                // the columns right of k + 1
                int slo, shi;
                srange(w, 0, tk1, slo, shi);
                la_update_reg<RT>(acc, c_slot3[w], slo, shi, k, S, dq, lr, lk);
                la_update_lds(S, NREG, NREG, tk1, w, k, dq, lr, lk);
            }
            __syncthreads();
            const long long te = __builtin_amdgcn_s_memtime();
            ph[0] += tb1 - ts;
            ph[1] += te - tb1;
        }
        tot += __builtin_amdgcn_s_memtime() - t0;
    }
    if (threadIdx.x == 0) cyc[blockIdx.x] = tot;
    if (threadIdx.x == 0 && blockIdx.x == 0)
        for (int i = 0; i < 4; ++i) cyc[4096 + i] = ph[i];
    if (blockIdx.x == 0 && w0 > 0) {
#pragma unroll
        for (int s = 0; s < RT; ++s) {
            const int t = 3 * s + w0 - 1;
            int I = 0, J = 0;
            tdecode(t < NREG ? t : 0, I, J);
            if (t < NREG) {
#pragma unroll
                for (int r = 0; r < 4; ++r) Lout[(16 * I + lk + 4 * r) * 256 + 16 * J + lr] = acc[s][r];
            }
        }
        for (int t = NREG + w0 - 1; t < NTILE; t += 3) {
            int I, J;
            tdecode(t, I, J);
            const ldouble* T = S + (t - NREG) * TS;
#pragma unroll
            for (int r = 0; r < 4; ++r) Lout[(16 * I + lk + 4 * r) * 256 + 16 * J + lr] = T[lr * CS + lk + 4 * r];
        }
    }
}

// v_mfma_f64_16x16x4_f64 issue rate with one wave per SIMD: CH independent accumulator
// chains, 64 instructions per chain
template <int CH>
__global__ __launch_bounds__(256, 1) void mfma_rate(double* out, long long* cyc) {
    double4v acc[CH];
#pragma unroll
    for (int c = 0; c < CH; ++c) acc[c] = double4v{0.0, 0.0, 0.0, 0.0};
    const double a = 1.0 + threadIdx.x * 1e-3, b = 0.5 - threadIdx.x * 1e-4;
    __syncthreads();
    const long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < 64; ++i)
#pragma unroll
        for (int c = 0; c < CH; ++c) acc[c] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[c], 0, 0, 0);
    double s = 0.0;
#pragma unroll
    for (int c = 0; c < CH; ++c) s += acc[c][0] + acc[c][3];
    asm volatile("s_nop 0" ::"v"(s));   // the stamp after the chains' results
    const long long t1 = __builtin_amdgcn_s_memtime();
    out[threadIdx.x] = s;
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

// The shipped factorisation (csrc/scpqp_kernel.h cholesky) on c3's plan: packed factor
// in the global workspace, RMAX 4, the grouped MFMA trailing update, two workgroups
// per CU (the dynamic LDS is sized like the c3 plan's, 69 KB, so that no more fit).
struct PLayG {
    static constexpr int RMAX = 4;
    static constexpr bool HGLOBAL = true;
    static constexpr int OCCV = 2;
    gdouble* H;
    ldouble *dinv, *red;
    int n, lead;
};

__global__ __launch_bounds__(256, 2) void shipped_factor(const double* Kp, double* wsp, double* dout, long long* cyc,
                                                          int reps) {
    PLayG L;
    const int hsz = pad2(roff(NN + 1) + 16);
    L.H = (gdouble*)wsp + (size_t)blockIdx.x * hsz;
    ldouble* sm = (ldouble*)smem_;
    L.red = sm + 2;
    L.dinv = L.red + red_size(true);
    L.n = NN;
    L.lead = lead_wave_elect((lint*)(L.red + kLeadSlot));
    long long tot = 0;
    bool ok = true;
    for (int r = 0; r < reps; ++r) {
        for (int e = threadIdx.x; e < hsz; e += 256) L.H[e] = Kp[e];   // packed rows (roff)
        __syncthreads();
        const long long t0 = __builtin_amdgcn_s_memtime();
        ok = cholesky(L);
        tot += __builtin_amdgcn_s_memtime() - t0;
        __syncthreads();
    }
    if (threadIdx.x == 0) cyc[blockIdx.x] = ok ? tot : -1;
    if (blockIdx.x == 0)
        for (int i = threadIdx.x; i < NN; i += 256) dout[i] = L.dinv[i];
}
}  // namespace

#define CHECK(x)                                                                          \
    do {                                                                                  \
        hipError_t e_ = (x);                                                              \
        if (e_ != hipSuccess) {                                                           \
            printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
            exit(1);                                                                      \
        }                                                                                 \
    } while (0)

template <int RT>
static void run_onchip(const std::vector<double>& K, double* dK, double* dL, long long* dc, int grid, int reps,
                       const std::vector<double>& Lref) {
    const int nreg = std::min(NTILE, 4 * RT);
    int nP = 0;
    for (int t = 0; t < nreg; ++t) {
        int I, J;
        tdecode(t, I, J);
        nP = std::max(nP, TN - I);
    }
    const int pbase = (NTILE - nreg) * TS, dbase = pbase + nP * TS;
    int slot[4][32], base[TN][TN] = {};
    for (int w = 0; w < 4; ++w)
        for (int q = 0; q < 32; ++q) {
            int I = 0, J = 0;
            const int t = 4 * q + w;
            if (q < RT && t < nreg) tdecode(t, I, J);
            slot[w][q] = (q < RT && t < nreg) ? (I | (J << 8)) : -1;
        }
    for (int I = 0; I < TN; ++I)
        for (int J = 0; J <= I; ++J) {
            const int t = tindex(I, J);
            base[I][J] = t < nreg ? pbase + (TN - 1 - I) * TS : (t - nreg) * TS;
        }
    CHECK(hipMemcpyToSymbol(HIP_SYMBOL(c_slot), slot, sizeof(slot)));
    CHECK(hipMemcpyToSymbol(HIP_SYMBOL(c_base), base, sizeof(base)));
    const size_t lds = (size_t)(dbase + 32) * 8;
    if (lds > 160 * 1024) {
        printf("on-chip RT=%d: %zu B of LDS does not fit\n", RT, lds);
        return;
    }
    auto k = onchip_factor<RT>;
    CHECK(hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    hipLaunchKernelGGL(k, dim3(grid), dim3(256), lds, 0, dK, dL, dc, 1, pbase, dbase);   // warm-up
    CHECK(hipEventRecord(e0));
    hipLaunchKernelGGL(k, dim3(grid), dim3(256), lds, 0, dK, dL, dc, reps, pbase, dbase);
    CHECK(hipEventRecord(e1));
    CHECK(hipDeviceSynchronize());
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    std::vector<long long> c(grid);
    std::vector<double> L(256 * 256);
    CHECK(hipMemcpy(c.data(), dc, grid * 8, hipMemcpyDeviceToHost));
    CHECK(hipMemcpy(L.data(), dL, L.size() * 8, hipMemcpyDeviceToHost));
    double err = 0;
    for (int i = 0; i < NN; ++i)
        for (int j = 0; j <= i; ++j) err = std::max(err, std::fabs(L[i * 256 + j] - Lref[i * NN + j]) / (1.0 + std::fabs(Lref[i * NN + j])));
    double mean = 0, mx = 0;
    for (long long v : c) mean += (double)v / grid, mx = std::max(mx, (double)v);
    std::vector<long long> p4(4);
    CHECK(hipMemcpy(p4.data(), dc + 4096, 32, hipMemcpyDeviceToHost));
    printf("on-chip  RT=%2d (%3d register tiles, LDS %6zu B) grid=%4d: %8.0f cycles/factorisation (max %8.0f), "
           "%9.0f factorisations/s (kernel %.3f ms), max |L - ref| %.1e\n",
           RT, std::min(NTILE, 4 * RT), lds, grid, mean / reps, mx / reps, grid * reps / (ms * 1e-3), ms, err);
    printf("         phases of workgroup 0 per factorisation: (a) to P %.0f, (b) diagonal tile %.0f, (c) panel rows %.0f, "
           "(d) trailing update %.0f cycles\n", (double)p4[0] / reps, (double)p4[1] / reps, (double)p4[2] / reps,
           (double)p4[3] / reps);
}

template <int RT>
static void run_onchip_la(double* dK, double* dL, long long* dc, int grid, int reps, const std::vector<double>& Lref) {
    const int nreg = std::min(NTILE, 3 * RT);
    int nP = 0;
    for (int t = 0; t < nreg; ++t) {
        int I, J;
        tdecode(t, I, J);
        nP = std::max(nP, TN - I);
    }
    const int pb0 = (NTILE - nreg) * TS, pb1 = pb0 + nP * TS, dbase = pb1 + nP * TS;
    const size_t lds = (size_t)(dbase + 64) * 8;
    if (lds > 160 * 1024) {
        printf("on-chip look-ahead RT=%d: %zu B of LDS does not fit\n", RT, lds);
        return;
    }
    int slot[4][32], base[TN][TN] = {};
    for (int w = 0; w < 4; ++w)
        for (int q = 0; q < 32; ++q) {
            int I = 0, J = 0;
            const int t = 3 * q + w - 1;
            const bool ok = w > 0 && q < RT && t < nreg;
            if (ok) tdecode(t, I, J);
            slot[w][q] = ok ? (I | (J << 8)) : -1;
        }
    for (int I = 0; I < TN; ++I)
        for (int J = 0; J <= I; ++J) {
            const int t = tindex(I, J);
            base[I][J] = t < nreg ? ((J & 1) ? pb1 : pb0) + (TN - 1 - I) * TS : (t - nreg) * TS;
        }
    CHECK(hipMemcpyToSymbol(HIP_SYMBOL(c_slot3), slot, sizeof(slot)));
    CHECK(hipMemcpyToSymbol(HIP_SYMBOL(c_base3), base, sizeof(base)));
    auto k = onchip_factor_la<RT>;
    CHECK(hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    hipLaunchKernelGGL(k, dim3(grid), dim3(256), lds, 0, dK, dL, dc, 1, pb0, pb1, dbase);
    CHECK(hipEventRecord(e0));
    hipLaunchKernelGGL(k, dim3(grid), dim3(256), lds, 0, dK, dL, dc, reps, pb0, pb1, dbase);
    CHECK(hipEventRecord(e1));
    CHECK(hipDeviceSynchronize());
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    std::vector<long long> c(grid), p4(4);
    std::vector<double> L(256 * 256);
    CHECK(hipMemcpy(c.data(), dc, grid * 8, hipMemcpyDeviceToHost));
    CHECK(hipMemcpy(p4.data(), dc + 4096, 32, hipMemcpyDeviceToHost));
    CHECK(hipMemcpy(L.data(), dL, L.size() * 8, hipMemcpyDeviceToHost));
    double err = 0;
    for (int i = 0; i < NN; ++i)
        for (int j = 0; j <= i; ++j) err = std::max(err, std::fabs(L[i * 256 + j] - Lref[i * NN + j]) / (1.0 + std::fabs(Lref[i * NN + j])));
    double mean = 0, mx = 0;
    for (long long v : c) mean += (double)v / grid, mx = std::max(mx, (double)v);
    printf("look-ahead RT=%2d (%3d register tiles, LDS %6zu B) grid=%4d: %8.0f cycles/factorisation (max %8.0f), "
           "%9.0f factorisations/s (kernel %.3f ms), max |L - ref| %.1e\n",
           RT, nreg, lds, grid, mean / reps, mx / reps, grid * reps / (ms * 1e-3), ms, err);
    printf("         per factorisation (workgroup 0): column k + 1 update + hand-over %.0f, panel phase %.0f "
           "(of which wave 0's panel %.0f) cycles\n", (double)p4[0] / reps, (double)p4[1] / reps, (double)p4[2] / reps);
}

static void run_shipped(double* dK, double* ws, double* dd, long long* dc, int grid,
                        int reps, const std::vector<double>& dref) {
    const size_t lds = 69 * 1024;
    auto k = shipped_factor;
    CHECK(hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    hipLaunchKernelGGL(k, dim3(grid), dim3(256), lds, 0, dK, ws, dd, dc, 1);
    CHECK(hipEventRecord(e0));
    hipLaunchKernelGGL(k, dim3(grid), dim3(256), lds, 0, dK, ws, dd, dc, reps);
    CHECK(hipEventRecord(e1));
    CHECK(hipDeviceSynchronize());
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    std::vector<long long> c(grid);
    std::vector<double> d(NN);
    CHECK(hipMemcpy(c.data(), dc, grid * 8, hipMemcpyDeviceToHost));
    CHECK(hipMemcpy(d.data(), dd, NN * 8, hipMemcpyDeviceToHost));
    double err = 0, mean = 0, mx = 0;
    bool failed = false;
    for (int i = 0; i < NN; ++i) err = std::max(err, std::fabs(d[i] - dref[i]) / std::fabs(dref[i]));
    for (long long v : c) failed |= v < 0, mean += (double)v / grid, mx = std::max(mx, (double)v);
    printf("shipped  (plan 2, workspace factor)                 grid=%4d: %8.0f cycles/factorisation (max %8.0f), "
           "%9.0f factorisations/s (kernel %.3f ms), max rel |1/D - ref| %.1e%s\n",
           grid, mean / reps, mx / reps, grid * reps / (ms * 1e-3), ms, err, failed ? " FAILED" : "");
}

int main() {
    // K = M M' / n + n I-like SPD test matrix with c3's order (the probe times the
    // factorisation only; the values do not change its operation count)
    std::vector<double> K(NN * NN), Lref(NN * NN), dref(NN);
    for (int i = 0; i < NN; ++i)
        for (int j = 0; j <= i; ++j)
            K[i * NN + j] = K[j * NN + i] = (i == j ? (double)NN : 0.0) + 0.5 * sin(0.3 * i + 0.6 * j) * sin(0.6 * i + 0.3 * j);
    {   // host L D L' (right-looking): L below the diagonal, D on it
        std::vector<double> A = K;
        for (int j = 0; j < NN; ++j) {
            const double D = A[j * NN + j];
            for (int i = j + 1; i < NN; ++i) {   // column j still unscaled on rows k < i
                const double l = A[i * NN + j] / D;
                for (int k = j + 1; k <= i; ++k) A[i * NN + k] -= l * A[k * NN + j];
            }
            for (int i = j + 1; i < NN; ++i) A[i * NN + j] /= D;
        }
        for (int i = 0; i < NN; ++i)
            for (int j = 0; j <= i; ++j) Lref[i * NN + j] = A[i * NN + j];
        for (int j = 0; j < NN; ++j) dref[j] = 1.0 / A[j * NN + j];
    }
    for (int t = 0; t < NTILE; ++t) {   // the tile order's decode is its inverse
        int I, J;
        tdecode(t, I, J);
        if (tindex(I, J) != t || I < J || J < 0 || I >= TN) {
            printf("tile decode broken at %d\n", t);
            return 1;
        }
    }
    int ncu = 0;
    CHECK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
    double *dK, *dL, *ws, *dd;
    long long* dc;
    CHECK(hipMalloc(&dK, K.size() * 8));
    CHECK(hipMalloc(&dL, 256 * 256 * 8));
    CHECK(hipMalloc(&dd, 512 * 8));
    CHECK(hipMalloc(&dc, 8192 * 8));
    const size_t hsz = pad2(roff(NN + 1) + 16);
    CHECK(hipMalloc(&ws, (size_t)2 * ncu * hsz * 8));
    CHECK(hipMemcpy(dK, K.data(), K.size() * 8, hipMemcpyHostToDevice));
    printf("CUs %d, n = %d\n", ncu, NN);
    {
        long long c1 = 0, c4 = 0, c16 = 0;
        hipLaunchKernelGGL(mfma_rate<1>, dim3(1), dim3(256), 0, 0, dd, dc);
        CHECK(hipMemcpy(&c1, dc, 8, hipMemcpyDeviceToHost));
        hipLaunchKernelGGL(mfma_rate<4>, dim3(1), dim3(256), 0, 0, dd, dc);
        CHECK(hipMemcpy(&c4, dc, 8, hipMemcpyDeviceToHost));
        hipLaunchKernelGGL(mfma_rate<16>, dim3(1), dim3(256), 0, 0, dd, dc);
        CHECK(hipMemcpy(&c16, dc, 8, hipMemcpyDeviceToHost));
        printf("v_mfma_f64_16x16x4_f64, one wave per SIMD: %.1f cycles per instruction on one chain, %.1f on 4 "
               "independent chains, %.1f on 16\n", c1 / 64.0, c4 / 256.0, c16 / 1024.0);
    }
    std::vector<double> Kp(hsz, 0.0);
    for (int i = 0; i < NN; ++i)
        for (int j = 0; j <= i; ++j) Kp[roff(i) + j] = K[i * NN + j];
    double* dKp;
    CHECK(hipMalloc(&dKp, hsz * 8));
    CHECK(hipMemcpy(dKp, Kp.data(), hsz * 8, hipMemcpyHostToDevice));
    for (int grid : {1, 2 * ncu}) run_shipped(dKp, ws, dd, dc, grid, grid == 1 ? 20 : 10, dref);
    for (int grid : {1, ncu}) {
        const int reps = grid == 1 ? 20 : 10;
        run_onchip<20>(K, dK, dL, dc, grid, reps, Lref);
        run_onchip<22>(K, dK, dL, dc, grid, reps, Lref);
        run_onchip<24>(K, dK, dL, dc, grid, reps, Lref);
        run_onchip_la<27>(dK, dL, dc, grid, reps, Lref);
    }
    return 0;
}
