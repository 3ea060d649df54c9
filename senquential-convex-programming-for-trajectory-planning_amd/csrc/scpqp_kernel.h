// scpqp_kernel.h — MI355X (gfx950) batched SCP-QP trajectory planner: the device code.
// (scpqp.hip: the C-ABI host side; kernels.hip: the kernel instantiations, in groups
// that build as separate translation units.)
//
// One workgroup (256 threads = 4 wave64) owns one problem at a time — one
// joint multi-vehicle QCQP of one MPC step — and runs the whole hot path of
// the reference for it without leaving the device:
//
//   K2  reference sampling            SampleReferTraj.py:8-122, MPC_Iter.py:35-43
//   K1  Jacobian + expm + prediction  Model.py:45-87, MPC_Iter.py:59-149
//   K3  constraint linearisation      SCP_controller.py:93-128 (factored, A.5)
//   K4  convexified QP                SCP_controller.py:118-150 (IPM + polish)
//   K3' QCQP evaluation               SCP_controller.py:215-265
//   K5  SCP loop + stopping rule      SCP_controller.py:40-49,74-197
//
// Problems are pulled from a device work counter, so workgroups that finish
// early (fewer SCP iterations, shorter horizon) immediately take the next one.
// Everything is fp64.  The per-problem state (KKT matrix, Toeplitz blocks,
// interior-point vectors) lives in LDS; when it does not fit (8 vehicles at
// Hp=30, or 4 vehicles at Hp=30), the KKT matrix and/or the constraint vectors
// move to a per-workgroup global workspace (template flags HG / VG).  All LDS
// arrays are addressed through address_space(3) pointers so every access is a
// ds_read/ds_write, never a flat access.
//
// The QP is solved in scaled variables (controls in units of
// uLim, every constraint row of unit norm) by a Mehrotra predictor-corrector
// interior point method on the normal equations
//     K = P + G' D G,   P = blkdiag(2 Phi0, 0),
// assembled from the Toeplitz structure:  K_uu = B'(2Q + W)B + diag,  with B
// the block-Toeplitz prediction matrix (g_m = C A^m B) and W block-diagonal
// per prediction step (2nVeh x 2nVeh blocks) — never the dense
// (nVeh-1) x nVeh x Hp x N x N tensors of QCQP_formulate.  The IPM is followed
// by an active-set polish (proximal method of multipliers on the identified
// active set, same assembly / Cholesky / triangular solves) that returns the
// exact minimiser when it certifies.

#pragma once

#include <hip/hip_runtime.h>

#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <new>
#include <type_traits>

#include "scpqp.h"

#define NT 256            // threads per workgroup (4 wave64)
#define TXD 16            // column stride of the 2-D thread grid
#define TYD (NT / TXD)    // row stride
#define NWAVE (NT / 64)
#define SCR_PER_WAVE 640

namespace {

// Diagnostic phase stamps (built only with -DSCPQP_PROF; never in the shipped kernel).
#ifdef SCPQP_PROF
__device__ unsigned long long g_prof[32];
__device__ unsigned long long g_ptime[8192 * 2];   // per-problem [start, end] (100 MHz realtime)
#define PROF_T0() unsigned long long _pt = __builtin_amdgcn_s_memtime()
#define PROF_ACC(cat)                                                              \
    do {                                                                           \
        unsigned long long _t1 = __builtin_amdgcn_s_memtime();                      \
        if (threadIdx.x == 0) atomicAdd(&g_prof[cat], _t1 - _pt);                   \
        _pt = _t1;                                                                 \
    } while (0)
// stamps inside code that only the lead wave runs (panel, triangular solves):
// counted from that wave's lane 0, whichever wave leads
#define PROF_ACC_LEAD(cat)                                                         \
    do {                                                                           \
        unsigned long long _t1 = __builtin_amdgcn_s_memtime();                      \
        if ((threadIdx.x & 63) == 0) atomicAdd(&g_prof[cat], _t1 - _pt);            \
        _pt = _t1;                                                                 \
    } while (0)
#else
#define PROF_T0() (void)0
#define PROF_ACC(cat) (void)0
#define PROF_ACC_LEAD(cat) (void)0
#endif
// Fine-grained stamps inside the factorisation (panel sub-phases, barrier waits):
// only with -DSCPQP_PROF_FINE, since their atomics perturb whole-batch timelines.
#if defined(SCPQP_PROF) && defined(SCPQP_PROF_FINE)
#define PROF_T0_FINE() PROF_T0()
#define PROF_ACC_FINE(cat) PROF_ACC_LEAD(cat)
#define PROF_ACC_FINE0(cat) PROF_ACC(cat)
#else
#define PROF_T0_FINE() (void)0
#define PROF_ACC_FINE(cat) (void)0
#define PROF_ACC_FINE0(cat) (void)0
#endif

typedef __attribute__((address_space(3))) double ldouble;
typedef __attribute__((address_space(3))) int lint;
typedef __attribute__((address_space(1))) int gint;
typedef __attribute__((address_space(1))) double gdouble;
typedef double double2v __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) double2v ldouble2;
typedef __attribute__((address_space(1))) double2v gdouble2;

// 16-byte loads (ds_read_b128 / global_load_dwordx4); callers pass even offsets
__device__ __forceinline__ double2v ld2(const ldouble* p) { return *(const ldouble2*)p; }
__device__ __forceinline__ void st2(ldouble* p, double2v v) { *(ldouble2*)p = v; }
__device__ __forceinline__ void st2(gdouble* p, double2v v) { *(gdouble2*)p = v; }
__device__ __forceinline__ double2v ld2(const gdouble* p) { return *(const gdouble2*)p; }

// ---------------------------------------------------------------------------
// Parameters (device copy of scpqp_params with derived constants)
// ---------------------------------------------------------------------------
struct DevParams {
    int nV, hpMax, nO, maxPts;
    int maxScp, maxIpm, nRefine, flags;
    double dt, uLim, ctol, deltaTol, slackW, ipmTol, polDelta, polRho;
    double Lf[SCPQP_MAX_VEH], Lr[SCPQP_MAX_VEH], Q[SCPQP_MAX_VEH], Qf[SCPQP_MAX_VEH],
        R[SCPQP_MAX_VEH];
    double D2veh[SCPQP_MAX_VEH * SCPQP_MAX_VEH];   // (dsafe + dsafeExtra)^2
    double D2obs[SCPQP_MAX_VEH * SCPQP_MAX_OBST];
    double poly[SCPQP_MAX_VEH * SCPQP_MAX_REFPTS * 2];
    int npts[SCPQP_MAX_VEH];
};

enum Mode { MODE_SOLVE = 0, MODE_LINEARIZE = 1, MODE_EVALUATE = 2, MODE_SAMPLE = 3 };

struct KArgs {
    const DevParams* P;
    int B, mode, maxScp, pad0;
    const double *x0, *u0, *ec, *obst, *refIn, *uWarm, *uEval;
    const int* hp;
    double *uOut, *trajOut, *obj, *maxv, *sumv;
    int *status, *nscp, *nipm, *feas, *npol, *nref, *nwarm;
    double *Ad, *Bd, *Ed, *gOut, *p0Out, *psiOut, *refOut;
    double *cveh, *cobs;
    double* trace;
    double* ws;
    long long wsStride;
    int* counter;
    const int* perm;   // optional: work item w -> problem perm[w] (longest horizons first)
};
// The kernel argument block, addressed in the constant (kernarg) address space:
// out-of-line functions take it by pointer without the copy to private memory
// that taking the address of a by-value kernel parameter would force.
typedef __attribute__((address_space(4))) const KArgs cKArgs;
// the parameter block is written once before the launch: read it through the
// constant address space so its fields come in as scalar loads
typedef __attribute__((address_space(4))) const DevParams cParams;


// ---------------------------------------------------------------------------
// Memory plan: integer offsets (doubles).  Persistent LDS arrays first, then a
// union region used by the setup scratch (expm) and, during the solve, by the
// KKT matrix, the W~ blocks and the 9 constraint-space vectors (those marked
// global go to the per-workgroup workspace instead).  Sizes use hp_max;
// indexing uses the problem's own horizon, so mixed horizons share a launch.
// ---------------------------------------------------------------------------
__host__ __device__ inline int pad2(int x) { return (x + 1) & ~1; }

// doubles per SCP iteration of the optional trace (scpqp.h, scpqp_batch_out.trace):
// a header of kTraceHdr, then u_lin, u and the factored rows
constexpr int kTraceHdr = 10;
__host__ __device__ inline int trace_stride(int V, int O, int Hm) {
    const int N = V * Hm, m = V * (V - 1) / 2 * Hm + V * O * Hm;
    return pad2(kTraceHdr + 2 * N + 4 * m);
}

// Packed lower-triangular storage of the KKT matrix: row i holds columns 0..i,
// padded to an even length so every row starts 16-byte aligned.
__host__ __device__ __forceinline__ int roff(int i) { return i * (i + 1) / 2 + ((i + 1) >> 1); }

// The reduction / slot area `red` of a plan (doubles): [0, 48) the three partial-sum
// buffers of block_reduce4, [0, 64) also the factorisation's look-ahead rows (ldbuf; no
// reduction runs inside the factorisation), then single slots, then the pivots.
constexpr int kRedFlag = 64;    // factorisation failure flag, 2 ints [step parity]
constexpr int kIdlSlot = 65;    // 1 / polish delta of the current polish round
constexpr int kWorkSlot = 66;   // the problem index taken from the work queue (int)
constexpr int kLeadSlot = 67;   // lead election (2 ints)
constexpr int kOrSlot = 68;     // workgroup OR of the sampler's quirk flags (int)
constexpr int kPivSlot = 72;    // pivots [step mod 2G][CB] (G = 4 panels per group on
                                // workspace factors, else 1; CB = 8)
__host__ __device__ constexpr int red_size(bool hG) { return kPivSlot + 2 * (hG ? 4 : 1) * 8; }
// the lean plan 1 (W~ blocks and constraint rows in the workspace beside the vectors) at
// two workgroups per CU (c5, Hp 30), or four (the round-6 c2 residency experiment)
__host__ __device__ constexpr bool lean_plan(bool hG, bool vG, int occ) { return !hG && vG && (occ == 2 || occ == 4); }

struct Off {
    int x0, u0, ec, g, p0, ref, ob, ub, pb, ya, yb, qs, rowE, rowW, rowH, rinfo;
    int z, dz, rhs, rd, dinv, red, scr;
    int H, Wt, vec;     // H and vec in LDS (after persist) or workspace, see hG / vG
    int persist, uni, ws;
    int ldAlloc, mcAlloc;
};

// lean (plan 1 at two workgroups per CU, OCC = 2): the W~ blocks and the constraint-row
// arrays go to the workspace as well, so that a factor of up to ~7.6k entries (4
// vehicles at Hp 30) stays in LDS with two workgroups per CU (= Lay::LEAN)
__host__ __device__ inline Off plan_offsets(int V, int O, int Hm, bool hG, bool vG, bool lean = false) {
    const int N = V * Hm, n = N + 1, m = V * (V - 1) / 2 * Hm + V * O * Hm;
    const int mc = m + 2 * N + 1, ld = n + ((6 - n % 4) % 4), nb = V * (V + 1) / 2;
    Off f;
#ifdef SCPQP_DIAG_REDUCE_CHECK
    int p = 2;   // smem_[0]: the reduction-buffer check's slot (bar)
#else
    int p = 0;
#endif
    f.x0 = p; p += pad2(6 * V);
    f.u0 = p; p += pad2(V);
    f.ec = p; p += pad2(2 * V);
    f.g = p; p += pad2(2 * N);
    f.p0 = p; p += pad2(2 * N);
    f.ref = p; p += pad2(2 * N);
    f.ob = p; p += pad2(2 * O * Hm);
    f.ub = p; p += pad2(N);
    f.pb = p; p += pad2(2 * N);
    f.ya = p; p += pad2(2 * N);
    f.yb = p; p += pad2(2 * N);
    f.qs = p; p += pad2(N);
    int w = 0;
    int& rp = lean ? w : p;   // constraint-row arrays: LDS, or the workspace (lean)
    f.rowE = rp; rp += pad2(2 * m);
    f.rowW = rp; rp += pad2(m);
    f.rowH = rp; rp += pad2(m);
    f.rinfo = rp; rp += pad2((m + 1) / 2);
    f.z = p; p += pad2(n);
    f.dz = p; p += pad2(n);
    f.rhs = p; p += pad2(n);
    f.rd = p; p += pad2(n);
    f.dinv = p; p += pad2(n);
    f.red = p; p += red_size(hG);   // kRedFlag ... kPivSlot
    f.persist = p;
    f.scr = p;
    int u = 0;
    // packed K plus one spare row (row n: target of the predicate-free tile stores)
    if (hG) { f.H = w; w += pad2(roff(n + 1) + 16); } else { f.H = p + u; u += pad2(roff(n + 1) + 16); }
    const int setup = NWAVE * SCR_PER_WAVE;
    // plan 2 with constraint-row arrays at least as large as the setup scratch (8
    // vehicles at Hp 30): the W~ blocks go to the workspace as well, and the setup
    // scratch (expm, dead before the first linearisation) shares the row arrays, so
    // the union is empty and two workgroups fit per CU
    const bool wG = (hG && vG && (n + 63) / 64 == 4) || lean;   // = Lay::WGLOBAL
    const bool rows_scr = wG && !lean && f.rinfo + pad2((m + 1) / 2) - f.rowE >= setup;
    if (wG) { f.Wt = w; w += pad2(4 * Hm * nb); } else { f.Wt = p + u; u += pad2(4 * Hm * nb); }
    if (vG) { f.vec = w; w += 9 * pad2(mc); } else { f.vec = p + u; u += 9 * pad2(mc); }
    f.uni = u > setup ? u : setup;
    if (rows_scr) {
        f.scr = f.rowE;
        f.uni = 0;
    }
    f.ws = w;
    f.ldAlloc = ld;
    f.mcAlloc = pad2(mc);
    return f;
}

template <bool HG, bool VG, int RM, int OCC>
struct Lay {
    static constexpr int RMAX = RM;   // row slots of the triangular solves (n <= 64 RM)
    static constexpr bool HGLOBAL = HG;   // the factor lives in the global workspace
    static constexpr int OCCV = OCC;      // workgroups per CU the registers are budgeted for
    using HT = typename std::conditional<HG, gdouble, ldouble>::type;
    using VT = typename std::conditional<VG, gdouble, ldouble>::type;
    int V, O, Hb, N, n, m, mc, ld, mp, nb;
    int lead;   // the wave that runs the serial parts (panel, triangular solves)
    ldouble *x0, *u0, *ec, *g, *p0, *ref, *ob, *ub, *pb, *ya, *yb, *qs;
    ldouble *z, *dz, *rhs, *rd, *dinv, *red, *scr;
    // lean plan 1 (two workgroups per CU): W~ and the constraint rows in the workspace
    static constexpr bool LEAN = lean_plan(HG, VG, OCC);
    // W~ blocks: in the workspace on plan 2 for factors of 4 row slots (plan_offsets)
    static constexpr bool WGLOBAL = (HG && VG && RM == 4) || LEAN;
    using WT = typename std::conditional<WGLOBAL, gdouble, ldouble>::type;
    using RT = typename std::conditional<LEAN, gdouble, ldouble>::type;
    using RIT = typename std::conditional<LEAN, gint, lint>::type;
    RT *rowE, *rowW, *rowH;
    RIT* rinfo;
    WT* Wt;
    HT* H;
    VT *s, *lam, *ds, *dl, *rp, *dd, *sa, *la, *tv;
};

// Problem shapes compiled as constants (template SH): the vehicle count, obstacle
// count and horizon of the BASELINE configurations, so that every loop bound,
// index division and LDS offset built from them folds at compile time (vehicle
// loops unrolled, Toeplitz trip counts known).  0 = runtime shape (any problem);
// a fixed horizon is used only when every problem of the launch has hp = hp_max.
// H: the problem's horizon; HM: the slot horizon the layout is planned for (hp_max).
// Shapes 4-6 are c5's horizon classes: the mixed-horizon kernel (shape 2) runs each
// problem's QPs with its horizon compiled in, in the launch's hp_max layout (round 5).
struct ShapeC {
    int V, O, H, HM;
};
__host__ __device__ constexpr ShapeC shape_c(int sh) {
    return sh == 1 ? ShapeC{4, 0, 20, 20}     // c2 / c4: 4 vehicles, Hp 20
         : sh == 2 ? ShapeC{4, 0, 0, 0}       // c5: 4 vehicles, mixed horizons
         : sh == 3 ? ShapeC{8, 0, 30, 30}     // c3: 8 vehicles, Hp 30
         : sh == 4 ? ShapeC{4, 0, 10, 0}      // c5 classes (QP solves of shape 2)
         : sh == 5 ? ShapeC{4, 0, 20, 0}
         : sh == 6 ? ShapeC{4, 0, 30, 0}
                   : ShapeC{0, 0, 0, 0};
}
template <int SH>
__host__ __device__ __forceinline__ int shapeV(int v) { return shape_c(SH).V ? shape_c(SH).V : v; }
template <int SH>
__host__ __device__ __forceinline__ int shapeO(int o) { return shape_c(SH).V ? shape_c(SH).O : o; }
template <int SH>
__host__ __device__ __forceinline__ int shapeH(int h) { return shape_c(SH).H ? shape_c(SH).H : h; }
template <int SH>
__host__ __device__ __forceinline__ int shapeHM(int h) { return shape_c(SH).HM ? shape_c(SH).HM : h; }

template <bool HG, bool VG, int RM, int OCC, int SH>
__device__ __forceinline__ Lay<HG, VG, RM, OCC> make_lay(ldouble* lds, gdouble* ws, const Off& f, int V,
                                                    int O, int Hb) {
    V = shapeV<SH>(V);
    O = shapeO<SH>(O);
    Hb = shapeH<SH>(Hb);
    Lay<HG, VG, RM, OCC> L;
    L.lead = 0;
    L.V = V; L.O = O; L.Hb = Hb; L.N = V * Hb; L.n = L.N + 1;
    L.mp = V * (V - 1) / 2 * Hb;
    L.m = L.mp + V * O * Hb;
    L.mc = L.m + 2 * L.N + 1;
    L.ld = f.ldAlloc;
    L.nb = V * (V + 1) / 2;
    L.x0 = lds + f.x0; L.u0 = lds + f.u0; L.ec = lds + f.ec; L.g = lds + f.g; L.p0 = lds + f.p0;
    L.ref = lds + f.ref; L.ob = lds + f.ob; L.ub = lds + f.ub; L.pb = lds + f.pb;
    L.ya = lds + f.ya; L.yb = lds + f.yb; L.qs = lds + f.qs;
    if constexpr (Lay<HG, VG, RM, OCC>::LEAN) {
        L.rowE = ws + f.rowE; L.rowW = ws + f.rowW; L.rowH = ws + f.rowH;
        L.rinfo = (gint*)(ws + f.rinfo);
    } else {
        L.rowE = lds + f.rowE; L.rowW = lds + f.rowW; L.rowH = lds + f.rowH;
        L.rinfo = (lint*)(lds + f.rinfo);
    }
    L.z = lds + f.z; L.dz = lds + f.dz;
    L.rhs = lds + f.rhs; L.rd = lds + f.rd; L.dinv = lds + f.dinv; L.red = lds + f.red;
    L.scr = lds + f.scr;
    if constexpr (Lay<HG, VG, RM, OCC>::WGLOBAL) L.Wt = ws + f.Wt; else L.Wt = lds + f.Wt;
    if constexpr (HG) L.H = ws + f.H; else L.H = lds + f.H;
    typename Lay<HG, VG, RM, OCC>::VT* vb;
    if constexpr (VG) vb = ws + f.vec; else vb = lds + f.vec;
    const int st = f.mcAlloc;
    L.s = vb; L.lam = vb + st; L.ds = vb + 2 * st; L.dl = vb + 3 * st; L.rp = vb + 4 * st;
    L.dd = vb + 5 * st; L.sa = vb + 6 * st; L.la = vb + 7 * st; L.tv = vb + 8 * st;
    return L;
}

extern __shared__ double smem_[];   // dynamic LDS (one problem's state)

// ---------------------------------------------------------------------------
// Small helpers
// ---------------------------------------------------------------------------
__device__ __forceinline__ unsigned long long readfirstlane_u64(unsigned long long v) {
    const unsigned lo = __builtin_amdgcn_readfirstlane(static_cast<unsigned>(v));
    const unsigned hi = __builtin_amdgcn_readfirstlane(static_cast<unsigned>(v >> 32));
    return (static_cast<unsigned long long>(hi) << 32) | lo;
}
__device__ __forceinline__ double readlane_d(double v, int lane) {
    long long bits = __double_as_longlong(v);
    int lo = __builtin_amdgcn_readlane(static_cast<int>(bits & 0xffffffffll), lane);
    int hi = __builtin_amdgcn_readlane(static_cast<int>(bits >> 32), lane);
    return __longlong_as_double((static_cast<long long>(hi) << 32) |
                                (static_cast<unsigned int>(lo)));
}

// Wave-wide reductions on DPP lane moves (VALU only; no LDS round trip as
// with ds_bpermute): quad xor 1 / xor 2, half-row and row mirrors combine 16
// lanes, then row_bcast:15 / row_bcast:31 carry rows 0..2 into lane 63.
template <int CTRL, int RMASK>
__device__ __forceinline__ double dpp_d(double v, double old) {
    const long long b = __double_as_longlong(v), o = __double_as_longlong(old);
    const int lo = __builtin_amdgcn_update_dpp((int)(o & 0xffffffffll), (int)(b & 0xffffffffll),
                                               CTRL, RMASK, 0xf, false);
    const int hi = __builtin_amdgcn_update_dpp((int)(o >> 32), (int)(b >> 32), CTRL, RMASK, 0xf,
                                               false);
    return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}
template <bool MAX>
__device__ __forceinline__ double wave_reduce(double v) {
    const double id = MAX ? -INFINITY : 0.0;
    auto op = [](double a, double b) { return MAX ? fmax(a, b) : a + b; };
    v = op(v, dpp_d<0xb1, 0xf>(v, id));    // quad_perm [1,0,3,2]
    v = op(v, dpp_d<0x4e, 0xf>(v, id));    // quad_perm [2,3,0,1]
    v = op(v, dpp_d<0x141, 0xf>(v, id));   // row_half_mirror
    v = op(v, dpp_d<0x140, 0xf>(v, id));   // row_mirror
    v = op(v, dpp_d<0x142, 0xa>(v, id));   // row_bcast:15 -> rows 1, 3
    v = op(v, dpp_d<0x143, 0xc>(v, id));   // row_bcast:31 -> rows 2, 3
    return readlane_d(v, 63);
}
__device__ __forceinline__ double wave_sum(double v) { return wave_reduce<false>(v); }
__device__ __forceinline__ double wave_max(double v) { return wave_reduce<true>(v); }

// Workgroup barrier.  Diagnostic build -DSCPQP_DIAG_REDUCE_CHECK: thread 0 also records
// that a barrier ran since the last block reduction (block_reduce4's buffer check), in the
// first slot of the dynamic LDS, which that build's plans reserve (plan_offsets).  (A
// static __shared__ variable beside the dynamic LDS, the first form of this check, faulted
// on the device: the plans assume the dynamic LDS starts at offset 0.)
#ifdef SCPQP_DIAG_REDUCE_CHECK
// [reductions checked, reductions whose buffer equals the previous reduction's with no
// barrier between them] (read by scpqp_diag_reduce_check)
__device__ unsigned g_redchk[2];
__device__ __forceinline__ lint& redchk_last() { return ((lint*)smem_)[0]; }
__device__ __forceinline__ void bar() {
    __syncthreads();
    if (threadIdx.x == 0) redchk_last() = -1;
}
#else
__device__ __forceinline__ void bar() { __syncthreads(); }
#endif

// Reduce four values across the workgroup; bit q of maxmask: max, else sum.
// NQ: number of leading slots in use (the rest are left untouched).
// BUF: which of three 16-slot buffers (red[16 BUF, 16 BUF + 16)) carries the partial
// sums.  One barrier (round 5; two before): a wave may write its partials while a
// slower wave still reads the previous reduction's, so two reductions that follow each
// other with no barrier between them use different buffers (DESIGN §3 lists the pairs;
// the SCPQP_DIAG_REDUCE_CHECK build counts every violation of that rule at run time,
// and a -DSCPQP_DIAG_REDUCE2 build, a barrier before the partials are written, gives
// the bitwise reference for the one-barrier form).
template <int NQ = 4, int BUF = 0>
__device__ __forceinline__ void block_reduce4(double (&v)[4], int maxmask, ldouble* red) {
    static_assert(BUF >= 0 && BUF < 3, "three partial-sum buffers in red[0, 48)");
    const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
    red += 16 * BUF;
#pragma unroll
    for (int q = 0; q < NQ; ++q) v[q] = (maxmask >> q & 1) ? wave_max(v[q]) : wave_sum(v[q]);
#ifdef SCPQP_DIAG_REDUCE2
    __syncthreads();
#endif
#ifdef SCPQP_DIAG_REDUCE_CHECK
    if (threadIdx.x == 0) {
        atomicAdd(&g_redchk[0], 1u);
        if (redchk_last() == BUF) atomicAdd(&g_redchk[1], 1u);
    }
#endif
    if (l == 0) {
#pragma unroll
        for (int q = 0; q < NQ; ++q) red[w * 4 + q] = v[q];
    }
    __syncthreads();
#ifdef SCPQP_DIAG_REDUCE_CHECK
    if (threadIdx.x == 0) redchk_last() = BUF;
#endif
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
        double r = red[q];
#pragma unroll
        for (int ww = 1; ww < NWAVE; ++ww)
            r = (maxmask >> q & 1) ? fmax(r, red[ww * 4 + q]) : r + red[ww * 4 + q];
        v[q] = r;
    }
}

// t -> (i, k) with t = i (i + 1) / 2 + k, 0 <= k <= i (lower-triangle enumeration)
__device__ __forceinline__ void tri_decode(int t, int& i, int& k) {
    int q = (int)((sqrtf(8.0f * (float)t + 1.0f) - 1.0f) * 0.5f);
    if ((q + 1) * (q + 2) / 2 <= t) ++q;
    if (q * (q + 1) / 2 > t) --q;
    i = q;
    k = t - q * (q + 1) / 2;
}

// Tile t -> (vehicle block a >= b, tile row lt, tile column mt) of the K_uu
// assembly, in order of increasing d = max(lt, mt): per d the V diagonal
// blocks' d + 1 tiles (lt = d, mt <= d), then the PV off-diagonal blocks'
// 2d + 1 tiles (lt = d, mt <= d; then mt = d, lt < d).
__device__ __forceinline__ void tile_decode(int t, int V, int PV, int& a, int& b, int& lt, int& mt) {
    int d = 0, base = 0;
    for (;;) {
        const int cnt = V * (d + 1) + PV * (2 * d + 1);
        if (t < base + cnt) break;
        base += cnt;
        ++d;
    }
    int r = t - base;
    if (r < V * (d + 1)) {
        a = b = r / (d + 1);
        lt = d;
        mt = r - a * (d + 1);
        return;
    }
    r -= V * (d + 1);
    const int pr = r / (2 * d + 1), q = r - pr * (2 * d + 1);
    int i_, k_;
    tri_decode(pr, i_, k_);
    a = i_ + 1;
    b = k_;
    if (q <= d) {
        lt = d;
        mt = q;
    } else {
        lt = q - (d + 1);
        mt = d;
    }
}

__device__ __forceinline__ int pair_index(int i, int j, int V) {
    return i * (2 * V - i - 1) / 2 + (j - i - 1);
}

// Row r -> (i, j, o, k): vehicle pair rows (i<j, k innermost) then obstacle
// rows (v, o, k) — the order of SCP_controller.py:97-114.
__device__ __forceinline__ void row_decode(int info, int& i, int& j, int& o, int& k) {
    i = info & 0xff;
    j = ((info >> 8) & 0xff) - 1;
    o = ((info >> 16) & 0xff) - 1;
    k = (info >> 24) & 0xff;
}

template <class LT>
__device__ __forceinline__ double hval(const LT& L, int i) {
    return i < L.m ? L.rowH[i] : (i < L.mc - 1 ? 1.0 : 0.0);
}

// ---------------------------------------------------------------------------
// Vehicle model (Model.py:45-87): entry (i, j) of the 8x8 expm argument
// [[Ac Bc Ec]; 0] computed per lane.
// ---------------------------------------------------------------------------
__device__ double jac_entry(const ldouble* x, double u, double Lf, double Lr, double n0, double n1,
                            int i, int j) {
    if (i >= 6) return 0.0;
    const double L = Lf + Lr, rho = Lr / L;
    const double v = x[3], psi = x[2], d = x[5];
    const double t = tan(d), sec2 = t * t + 1.0;
    const double kap = sqrt(rho * rho * t * t + 1.0);
    const double beta = atan(rho * t);
    const double th = psi + beta;
    const double cth = cos(th), sth = sin(th);
    // analytic Ac (Model.py:46-52)
    double a02 = -v * sth * kap, a03 = cth * kap;
    double a05 = rho * rho * v * cth * t * sec2 / kap - rho * v * sth * sec2 / kap;
    double a12 = v * cth * kap, a13 = sth * kap;
    double a15 = rho * v * cth * sec2 / kap + rho * rho * v * sth * t * sec2 / kap;
    double a23 = t / L, a25 = v * sec2 / L;
    if (j < 6) {
        if (i == 0) return j == 2 ? a02 : j == 3 ? a03 : j == 5 ? a05 : 0.0;
        if (i == 1) return j == 2 ? a12 : j == 3 ? a13 : j == 5 ? a15 : 0.0;
        if (i == 2) return j == 3 ? a23 : j == 5 ? a25 : 0.0;
        if (i == 3) return j == 4 ? 1.0 : 0.0;
        if (i == 5) return j == 5 ? -10.0 : 0.0;
        return 0.0;
    }
    if (j == 6) return i == 5 ? 10.0 : 0.0;   // Bc (Model.py:53)
    // Ec = f(x,u) - Ac x - Bc u   (Model.py:58), noise on dx[0], dx[1] (:84-86)
    const double vc = v * sqrt(1.0 + (rho * t) * (rho * t));
    if (i == 0) return (vc * cos(psi + beta) + n0) - (a02 * x[2] + a03 * x[3] + a05 * x[5]);
    if (i == 1) return (vc * sin(psi + beta) + n1) - (a12 * x[2] + a13 * x[3] + a15 * x[5]);
    if (i == 2) return vc * t * cos(beta) / L - (a23 * x[3] + a25 * x[5]);
    if (i == 3) return x[4] - x[4];
    if (i == 4) return 0.0;
    return (u - x[5]) / 0.1 - (-10.0 * x[5]) - 10.0 * u;
}

// ---------------------------------------------------------------------------
// Reference sampler (SampleReferTraj.py:8-122), one lane per vehicle.
// Quirks B.1 (alternation past the end) and B.3 (rear-axle speed) reproduced;
// B.2's float '^' (reference raises) is evaluated with '**' and flagged.
// ---------------------------------------------------------------------------
__device__ int sample_reference(const cParams& P, int v, double vx, double vy, double step,
                                int Hb, ldouble* out /* [Hb][2] */) {
    const auto* c = P.poly + v * P.maxPts * 2;
    const int np = P.npts[v];
    int flag = 0;
    // getShortestDistance: seeded with curve point 1, index 2 (quirk B.2)
    double xm = c[2], ym = c[3];
    double dmin = sqrt((vx - c[2]) * (vx - c[2]) + (vy - c[3]) * (vy - c[3]));
    int imin = 2;
    for (int j = 1; j < np; ++j) {
        const double x1 = c[2 * (j - 1)], y1 = c[2 * (j - 1) + 1], x2 = c[2 * j], y2 = c[2 * j + 1];
        const double bl = sqrt((x2 - x1) * (x2 - x1) + (y2 - y1) * (y2 - y1));
        double xp, yp, sd, lam;
        if (bl != 0.0) {
            const double xn = (x2 - x1) / bl, yn = (y2 - y1) / bl;
            const double x31 = vx - x1, y31 = vy - y1;
            const double dot = xn * x31 + yn * y31;
            sd = xn * y31 - yn * x31;
            xp = x1 + dot * xn;
            yp = y1 + dot * yn;
            lam = dot / bl;
        } else {
            sd = sqrt((vx - x1) * (vx - x1) + (vy - y1) * (vy - y1));
            lam = 0.0;
            xp = x1;
            yp = y1;
        }
        if ((0.0 < lam || j == 1) && (lam < 1.0 || j == np - 1)) {
            if (fabs(sd) < fabs(dmin)) {
                xm = xp; ym = yp; dmin = sd; imin = j;
            }
        } else {
            flag = 1;   // reference raises TypeError here (float ^ int)
            const double de = sqrt((vx - x2) * (vx - x2) + (vy - y2) * (vy - y2));
            if (de < fabs(dmin)) {
                xm = x2; ym = y2; dmin = (sd > 0.0) ? de : ((sd < 0.0) ? -de : 0.0); imin = j;
            }
        }
    }
    for (int i = 0; i + 1 < np; ++i) {
        const double dx = c[2 * i + 2] - c[2 * i], dy = c[2 * i + 3] - c[2 * i + 1];
        if (!(sqrt(dx * dx + dy * dy) > step)) flag = 1;   // SampleReferTraj.py:18-19 assert
    }
    int idx = imin;
    if (idx > np - 1) {   // vehicle exactly on the endpoint: reference raises IndexError
        idx = np - 1;
        flag = 1;
    }
    double cx = xm, cy = ym;
    for (int i = 0; i < Hb; ++i) {
        const double ex = c[2 * idx], ey = c[2 * idx + 1];
        const double rem = sqrt((cx - ex) * (cx - ex) + (cy - ey) * (cy - ey));
        if (rem > step || idx == np) {
            const double dx = ex - c[2 * idx - 2], dy = ey - c[2 * idx - 1];
            const double nr = sqrt(dx * dx + dy * dy);
            cx = cx + step * (dx / nr);
            cy = cy + step * (dy / nr);
        } else {
            cx = ex; cy = ey;
            idx = idx < np - 1 ? idx : np - 1;
            const double dx = c[2 * idx] - c[2 * idx - 2], dy = c[2 * idx + 1] - c[2 * idx - 1];
            const double nr = sqrt(dx * dx + dy * dy);
            cx = cx + (step - rem) * (dx / nr);
            cy = cy + (step - rem) * (dy / nr);
        }
        out[2 * i] = cx;
        out[2 * i + 1] = cy;
    }
    return flag;
}

// ---------------------------------------------------------------------------
// 8x8 matrix exponential, one wave per vehicle, lane = entry (i = lane>>3,
// j = lane&7).  Pade-13 with scaling and squaring (Higham 2005; the algorithm
// family of scipy.linalg.expm used at MPC_Iter.py:106,111).  The single 8x8
// expm(dt [[Ac Bc Ec];0]) gives Ad, Bd and Ed at once.
// All waves execute the same barrier sequence (`act` masks the work).
// ---------------------------------------------------------------------------
__device__ __forceinline__ double mm_entry(const ldouble* A, const ldouble* B, int i, int j) {
    double acc = 0.0;
#pragma unroll
    for (int k = 0; k < 8; ++k) acc += A[i * 8 + k] * B[k * 8 + j];
    return acc;
}

__device__ void expm8(ldouble* scr, bool act, ldouble* red) {
    const int lane = threadIdx.x & 63, i = lane >> 3, j = lane & 7;
    ldouble* M = scr;
    ldouble* A = scr + 64;
    ldouble* A2 = scr + 128;
    ldouble* A4 = scr + 192;
    ldouble* A6 = scr + 256;
    ldouble* T1 = scr + 320;
    ldouble* T2 = scr + 384;
    ldouble* U = scr + 448;
    ldouble* Vv = scr + 512;
    const double b0 = 64764752532480000.0, b1 = 32382376266240000.0, b2 = 7771770303897600.0,
                 b3 = 1187353796428800.0, b4 = 129060195264000.0, b5 = 10559470521600.0,
                 b6 = 670442572800.0, b7 = 33522128640.0, b8 = 1323241920.0, b9 = 40840800.0,
                 b10 = 960960.0, b11 = 16380.0, b12 = 182.0, b13 = 1.0;
    const double theta13 = 5.371920351148152;
    double cs = 0.0;
    if (act) {
#pragma unroll
        for (int r = 0; r < 8; ++r) cs += fabs(M[r * 8 + j]);
    }
    const double nrm = wave_max(cs);
    int s = 0;
    if (nrm > theta13) s = (int)ceil(log2(nrm / theta13));
    if (act) A[lane] = ldexp(M[lane], -s);
    // squaring count must be uniform across the workgroup (barriers below)
    if (lane == 0) red[threadIdx.x >> 6] = act ? (double)s : 0.0;
    bar();
    int smax = 0;
#pragma unroll
    for (int ww = 0; ww < NWAVE; ++ww) smax = max(smax, (int)red[ww]);
    if (act) A2[lane] = mm_entry(A, A, i, j);
    bar();
    if (act) A4[lane] = mm_entry(A2, A2, i, j);
    bar();
    if (act) A6[lane] = mm_entry(A4, A2, i, j);
    bar();
    if (act) {
        T1[lane] = b13 * A6[lane] + b11 * A4[lane] + b9 * A2[lane];
        T2[lane] = b12 * A6[lane] + b10 * A4[lane] + b8 * A2[lane];
    }
    bar();
    const double id = (i == j) ? 1.0 : 0.0;
    if (act) {
        U[lane] = mm_entry(A6, T1, i, j) + b7 * A6[lane] + b5 * A4[lane] + b3 * A2[lane] + b1 * id;
        Vv[lane] = mm_entry(A6, T2, i, j) + b6 * A6[lane] + b4 * A4[lane] + b2 * A2[lane] + b0 * id;
    }
    bar();
    if (act) T1[lane] = mm_entry(A, U, i, j);   // U = A * U2
    bar();
    // augmented [V-U | V+U] (8 x 16) in aug = scr[0..127]
    ldouble* aug = scr;
    if (act) {
        aug[i * 16 + j] = Vv[lane] - T1[lane];
        aug[i * 16 + 8 + j] = Vv[lane] + T1[lane];
    }
    bar();
    // Gauss-Jordan with partial pivoting (first maximal pivot, as LAPACK idamax)
    for (int k = 0; k < 8; ++k) {
        double key = -1.0;
        if (act && lane < 8 && lane >= k) key = fabs(aug[lane * 16 + k]);
        const double best = wave_max(key);
        unsigned long long ball = __ballot(act && lane < 8 && lane >= k && key == best);
        const int p = ball ? __ffsll((long long)ball) - 1 : k;
        bar();
        if (act && p != k && lane < 16) {
            const double t0 = aug[k * 16 + lane];
            aug[k * 16 + lane] = aug[p * 16 + lane];
            aug[p * 16 + lane] = t0;
        }
        bar();
        double nv0 = 0.0, nv1 = 0.0;
        if (act) {
            const double piv = aug[k * 16 + k];
            const double fi = aug[i * 16 + k];
            const double a0 = aug[i * 16 + j], a1 = aug[i * 16 + 8 + j];
            if (i == k) {
                nv0 = a0 / piv;
                nv1 = a1 / piv;
            } else {
                nv0 = a0 - fi * (aug[k * 16 + j] / piv);
                nv1 = a1 - fi * (aug[k * 16 + 8 + j] / piv);
            }
        }
        bar();
        if (act) {
            aug[i * 16 + j] = nv0;
            aug[i * 16 + 8 + j] = nv1;
        }
        bar();
    }
    // X = aug[:, 8:16] -> A (aliases aug rows 4..7: read, barrier, write); square s times
    {
        const double xv = act ? aug[i * 16 + 8 + j] : 0.0;
        bar();
        if (act) A[lane] = xv;
        bar();
    }
    for (int q = 0; q < smax; ++q) {
        const bool sq = act && q < s;
        const double v = sq ? mm_entry(A, A, i, j) : 0.0;
        bar();
        if (sq) A[lane] = v;
        bar();
    }
    // result in A (= scr + 64)
}

// ---------------------------------------------------------------------------
// Problem setup: inputs, reference sampling, per-vehicle linearisation
// (MPCclass, MPC_Iter.py:59-149), scaled cost gradient, row table.
// ---------------------------------------------------------------------------
template <class LT>
__device__ int setup_problem(const cKArgs& a, const cParams& P, const LT& L, int b) {
    const int tid = threadIdx.x, V = L.V, O = L.O, Hb = L.Hb, Hm = P.hpMax;
    for (int i = tid; i < 6 * V; i += NT) L.x0[i] = a.x0[(size_t)b * V * 6 + i];
    for (int i = tid; i < V; i += NT) L.u0[i] = a.u0 ? a.u0[(size_t)b * V + i] : 0.0;
    for (int i = tid; i < 2 * V; i += NT) L.ec[i] = a.ec ? a.ec[(size_t)b * V * 2 + i] : 0.0;
    for (int i = tid; i < O * 2 * Hb; i += NT) {
        const int o = i / (2 * Hb), c = (i / Hb) & 1, k = i % Hb;
        L.ob[(o * Hb + k) * 2 + c] = a.obst ? a.obst[(size_t)b * O * 2 * Hm + i] : 0.0;
    }
    bar();
    int sflag = 0;
    if (a.refIn) {
        for (int i = tid; i < Hb * 2 * V; i += NT) {
            const int k = i / (2 * V), c = (i / V) & 1, v = i % V;
            L.ref[(v * Hb + k) * 2 + c] = a.refIn[(size_t)b * Hm * 2 * V + i];
        }
    } else if (tid < V) {
        const ldouble* xv = L.x0 + 6 * tid;
        sflag = sample_reference(P, tid, xv[0], xv[1], xv[3] * P.dt, Hb, L.ref + tid * Hb * 2);
    }
    bar();
    if (a.mode == MODE_SAMPLE) return sflag;

    // per-vehicle linearisation, one wave per vehicle per round
    const int w = tid >> 6, lane = tid & 63;
    for (int r0 = 0; r0 < V; r0 += NWAVE) {
        const int v = r0 + w;
        const bool act = v < V;
        ldouble* scr = L.scr + w * SCR_PER_WAVE;
        if (act) {
            scr[lane] = P.dt * jac_entry(L.x0 + 6 * v, L.u0[v], P.Lf[v], P.Lr[v], L.ec[2 * v],
                                         L.ec[2 * v + 1], lane >> 3, lane & 7);
        }
        bar();
        expm8(scr, act, L.red);
        // Ad = X[0:6,0:6], Bd = X[0:6,6], Ed = X[0:6,7] (threshold 1e-30, MPC_Iter.py:87)
        double adrow[6];
        double bi = 0.0, ei = 0.0, xi = 0.0;
        const ldouble* X = scr + 64;
        const int comp = lane < 8 ? lane : lane - 8;   // lanes 0..5: state, 8..13: impulse
#pragma unroll
        for (int jj = 0; jj < 6; ++jj) adrow[jj] = 0.0;
        if (act && comp < 6 && lane < 16) {
#pragma unroll
            for (int jj = 0; jj < 6; ++jj) adrow[jj] = X[comp * 8 + jj];
            bi = X[comp * 8 + 6];
            ei = X[comp * 8 + 7];
            if (fabs(ei) <= 1e-30) ei = 0.0;
            xi = L.x0[6 * v + comp];
        }
        if (act && a.mode == MODE_LINEARIZE && lane < 6) {
            const size_t base = ((size_t)b * V + v);
            if (a.Ad)
#pragma unroll
                for (int jj = 0; jj < 6; ++jj) a.Ad[base * 36 + lane * 6 + jj] = adrow[jj];
            if (a.Bd) a.Bd[base * 6 + lane] = bi;
            if (a.Ed) a.Ed[base * 6 + lane] = ei;
        }
        // recursions: x_{k+1} = Ad x_k + Ed (p0_k = C x_{k+1});  b_{m+1} = Ad b_m (g_m = C b_m)
        double cur = (lane < 8) ? xi : bi;
        const double add = (lane < 8) ? ei : 0.0;
        const int base = lane < 8 ? 0 : 8;
        for (int k = 0; k < Hb; ++k) {
            if (lane >= 8 && lane < 10 && act) L.g[(v * Hb + k) * 2 + comp] = cur;
            double nxt = add;
#pragma unroll
            for (int jj = 0; jj < 6; ++jj) nxt += adrow[jj] * __shfl(cur, base + jj, 64);
            cur = nxt;
            if (lane < 2 && act) L.p0[(v * Hb + k) * 2 + lane] = cur;
        }
        bar();
    }
    // scaled cost gradient  qs = uLim * Psi0,  Psi0 = -2 calB' Q (ref - const)  (MPC_Iter.py:125)
    for (int e = tid; e < V * Hb; e += NT) {
        const int v = e / Hb, l = e % Hb;
        double acc = 0.0;
        for (int k = l; k < Hb; ++k) {
            const double qk = (k == Hb - 1) ? P.Qf[v] : P.Q[v];
            const ldouble* gg = L.g + (v * Hb + k - l) * 2;
            const double ex = L.ref[(v * Hb + k) * 2] - L.p0[(v * Hb + k) * 2];
            const double ey = L.ref[(v * Hb + k) * 2 + 1] - L.p0[(v * Hb + k) * 2 + 1];
            acc += qk * (gg[0] * ex + gg[1] * ey);
        }
        L.qs[e] = P.uLim * (-2.0 * acc);
    }
    // row table
    for (int r = tid; r < L.m; r += NT) {
        int i, j, o, k;
        if (r < L.mp) {
            const int pi = r / Hb;
            k = r % Hb;
            int ii = 0, rem = pi;
            while (rem >= V - 1 - ii) { rem -= V - 1 - ii; ++ii; }
            i = ii;
            j = ii + 1 + rem;
            o = -1;
        } else {
            const int ro = r - L.mp;
            const int vo = ro / Hb;
            k = ro % Hb;
            i = vo / O;
            o = vo % O;
            j = -1;
        }
        L.rinfo[r] = i | ((j + 1) << 8) | ((o + 1) << 16) | (k << 24);
    }
    bar();
    return sflag;
}

// Out-of-line setup: the trigonometry and expm constants stay out of the
// register allocation of the solve loop.
template <bool HG, bool VG, int RM, int OCC, int SH>
__device__ __noinline__ int setup_problem_ni(const cKArgs* ap, gdouble* ws, int b, int Hb) {
    // uniform arguments arrive in VGPRs: back to SGPRs (see uniform_ctx)
    ap = (const cKArgs*)readfirstlane_u64((unsigned long long)ap);
    ws = (gdouble*)readfirstlane_u64((unsigned long long)ws);
    b = __builtin_amdgcn_readfirstlane(b);
    Hb = __builtin_amdgcn_readfirstlane(Hb);
    const cKArgs& a = *ap;
    const cParams& P = *(const cParams*)a.P;
    const Off f = plan_offsets(shapeV<SH>(P.nV), shapeO<SH>(P.nO), shapeHM<SH>(P.hpMax), HG, VG, lean_plan(HG, VG, OCC));
    const Lay<HG, VG, RM, OCC> L = make_lay<HG, VG, RM, OCC, SH>((ldouble*)smem_, ws, f, P.nV, P.nO, Hb);
    return setup_problem(a, P, L, b);
}

// ---------------------------------------------------------------------------
// Structured linear operators (y-space = predicted-position space, [V][Hb][2])
// ---------------------------------------------------------------------------
// Toeplitz products over three lanes per output: an output's sum of up to Hb
// terms is split by term index mod 3 over lanes 3j, 3j+1, 3j+2 of a wave
// (21 outputs per wave, 84 per pass of the 256 threads) and recombined with
// two lane shuffles, so the longest serial chain is ceil(Hb / 3) terms and
// all four waves share the work (one lane per output used 80 of 256 threads
// with chains of up to Hb terms).  fn(e, sum) runs in the owner lane (s == 0).
constexpr int kSplit = 3, kPerWave = 21, kPerPass = kPerWave * NWAVE;
template <class TermSum, class Fn>
__device__ __forceinline__ void split3_outputs(int nout, TermSum part, Fn fn) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int j = lane / kSplit, sidx = lane - j * kSplit;
    for (int base = 0; base < nout; base += kPerPass) {
        const int e = base + w * kPerWave + j;
        const bool valid = lane < kSplit * kPerWave && e < nout;
        double2v acc = valid ? part(e, sidx) : double2v{0.0, 0.0};
        const double x1 = __shfl_down(acc.x, 1), y1 = __shfl_down(acc.y, 1);
        const double x2 = __shfl_down(acc.x, 2), y2 = __shfl_down(acc.y, 2);
        if (valid && sidx == 0) fn(e, double2v{acc.x + x1 + x2, acc.y + y1 + y2});
    }
}

// y[v][k] = sum_{l<=k} g[v][k-l] * x[v*Hb + l]     (calB x, MPC_Iter.py:146-147)
template <class LT, class PX, class PY>
__device__ __forceinline__ void toeplitz_apply(const LT& L, PX x, PY y) {
    split3_outputs(
        L.V * L.Hb,
        [&](int e, int sidx) {
            const int v = e / L.Hb, k = e - v * L.Hb;
            const ldouble* gv = L.g + v * L.Hb * 2;
            const int xb = v * L.Hb;
            double a0 = 0.0, a1 = 0.0;
            for (int l = sidx; l <= k; l += kSplit) {
                const double xl = x[xb + l];
                const double2v gl = ld2(gv + (k - l) * 2);
                a0 += gl.x * xl;
                a1 += gl.y * xl;
            }
            return double2v{a0, a1};
        },
        [&](int e, double2v r) { st2(y + 2 * e, r); });
}

// out(e, sum_{k>=l} g[v][k-l]' y[v][k]) for every e = v*Hb + l   (calB' y)
template <class LT, class PY, class Fn>
__device__ __forceinline__ void toeplitz_t_apply(const LT& L, PY y, Fn out) {
    split3_outputs(
        L.V * L.Hb,
        [&](int e, int sidx) {
            const int v = e / L.Hb, l = e - v * L.Hb;
            const ldouble* gv = L.g + v * L.Hb * 2;
            const int yb = v * L.Hb * 2;
            double acc = 0.0;
            for (int k = l + sidx; k < L.Hb; k += kSplit)
                acc += gv[(k - l) * 2] * y[yb + 2 * k] + gv[(k - l) * 2 + 1] * y[yb + 2 * k + 1];
            return double2v{acc, 0.0};
        },
        [&](int e, double2v r) { out(e, r.x); });
}

// sum over the rows incident to (v, k) of coef(r) * sigma * e_r  (2-vector)
template <class LT, class F>
__device__ __forceinline__ void incident_sum(const LT& L, int v, int k, F coef, double& s0,
                                            double& s1) {
    s0 = 0.0;
    s1 = 0.0;
    for (int w = 0; w < L.V; ++w) {
        if (w == v) continue;
        const int i = v < w ? v : w, j = v < w ? w : v;
        const int r = pair_index(i, j, L.V) * L.Hb + k;
        const double c = (v == i ? -1.0 : 1.0) * coef(r);
        s0 += c * L.rowE[2 * r];
        s1 += c * L.rowE[2 * r + 1];
    }
    for (int o = 0; o < L.O; ++o) {
        const int r = L.mp + (v * L.O + o) * L.Hb + k;
        const double c = -coef(r);
        s0 += c * L.rowE[2 * r];
        s1 += c * L.rowE[2 * r + 1];
    }
}

// (G x)_r given ya = calB x_u
template <class LT, class PX>
__device__ __forceinline__ double gx_row(const LT& L, PX xu, double xw, int r) {
    if (r < L.m) {
        int i, j, o, k;
        row_decode(L.rinfo[r], i, j, o, k);
        const double e0 = L.rowE[2 * r], e1 = L.rowE[2 * r + 1];
        double val = -(e0 * L.ya[(i * L.Hb + k) * 2] + e1 * L.ya[(i * L.Hb + k) * 2 + 1]);
        if (j >= 0) val += e0 * L.ya[(j * L.Hb + k) * 2] + e1 * L.ya[(j * L.Hb + k) * 2 + 1];
        return val + L.rowW[r] * xw;
    }
    if (r < L.m + L.N) return xu[r - L.m];
    if (r < L.m + 2 * L.N) return -xu[r - L.m - L.N];
    return -xw;
}

// G' t: fin(e, (G't)_e) for the u-part e < N (in the thread that owns e), omega part
// returned (uniform).  No barrier after the u-part: the caller's next barrier publishes it.
// BUF: the reduction's buffer (block_reduce4), chosen by the caller against the
// reduction before it.
template <int BUF, class LT, class PT, class Fin>
__device__ double gt_apply_fin(const LT& L, PT t, Fin fin) {
    const int tid = threadIdx.x;
    double wsum = 0.0;
    for (int e = tid; e < L.V * L.Hb; e += NT) {
        const int v = e / L.Hb, k = e % L.Hb;
        double s0, s1;
        incident_sum(L, v, k, [&](int r) { return t[r]; }, s0, s1);
        L.yb[2 * e] = s0;
        L.yb[2 * e + 1] = s1;
    }
    for (int r = tid; r < L.m; r += NT) wsum += t[r] * L.rowW[r];
    double red[4] = {wsum, 0.0, 0.0, 0.0};
    block_reduce4<1, BUF>(red, 0, L.red);   // barrier: yb visible afterwards
    toeplitz_t_apply(L, L.yb, [&](int e, double tt) { fin(e, tt + t[L.m + e] - t[L.m + L.N + e]); });
    return red[0] - t[L.mc - 1];
}

// ---------------------------------------------------------------------------
// Normal matrix assembly  K = P_s + rho I + G' diag(d) G   (lower triangle)
// ---------------------------------------------------------------------------
// K_uu lower triangle in TS x TS tiles (rows l0 .. l0+TS-1 of vehicle a x columns
// m0 .. m0+TS-1 of vehicle b, a >= b): K_(a,l),(b,l') = sum_k g_a,k-l' W~_ab,k
// g_b,k-l' over k >= max(l, l').  Per k one W~ block and TS g 2-vectors of each
// vehicle serve TS^2 entries; the g operands slide (row l0+i at step k uses the
// value row l0+i-1 used at step k-1), so a step loads one new g of each vehicle
// and one W~ block.  g indices below 0 read as zero, which gives each entry its
// own lower summation bound.  A tile's cost is its trip count Hb - TS max(lt, mt):
// tiles are enumerated by decreasing cost and dealt to the threads in snake
// order, so every thread gets about the same number of trips.
template <int TS, class LT, class PD>
__device__ __forceinline__ void assemble_tiles(const cParams& P, const LT& L, PD d, double rho) {
    const int tid = threadIdx.x, V = L.V, Hb = L.Hb, nb = L.nb, N = L.N;
    const double u2 = P.uLim * P.uLim;
    const int TH = (Hb + TS - 1) / TS, TD = TH * (TH + 1) / 2, TO = TH * TH;
    const int PV = V * (V - 1) / 2;
    const int ntile = V * TD + PV * TO;
    const double2v zero2 = {0.0, 0.0};
    for (int r0 = 0; r0 < ntile; r0 += NT) {
        const int t = r0 + (((r0 / NT) & 1) ? NT - 1 - tid : tid);
        if (t >= ntile) continue;
        int a_, b_, lt, mt;
        tile_decode(t, V, PV, a_, b_, lt, mt);
        const int l0 = TS * lt, m0 = TS * mt, k0 = l0 > m0 ? l0 : m0;
        const ldouble* ga = L.g + a_ * Hb * 2;
        const ldouble* gb = L.g + b_ * Hb * 2;
        const auto* W = L.Wt + 4 * (a_ * (a_ + 1) / 2 + b_);
        double2v av[TS], bv[TS];   // the window at step k0 - 1
#pragma unroll
        for (int i = 0; i < TS; ++i) {
            const int ia = k0 - 1 - l0 - i, ib = k0 - 1 - m0 - i;
            av[i] = ia >= 0 ? ld2(ga + 2 * ia) : zero2;
            bv[i] = ib >= 0 ? ld2(gb + 2 * ib) : zero2;
        }
        double c[TS][TS];
#pragma unroll
        for (int i = 0; i < TS; ++i)
#pragma unroll
            for (int j = 0; j < TS; ++j) c[i][j] = 0.0;
        // software pipeline: the next step's g and W~ loads are in flight while this
        // step's products run (the loop is LDS-latency-bound, not FMA-bound)
        double2v an = ld2(ga + 2 * (k0 - l0)), bn = ld2(gb + 2 * (k0 - m0));
        double2v wn0 = ld2(W + 4 * k0 * nb), wn1 = ld2(W + 4 * k0 * nb + 2);
        // two steps ahead where g / W~ come from the workspace (plan 2: c3 5.36k -> 5.54k
        // solves/s, profiles/r03_ab_prefetch.txt); one step for the LDS plans (c2, c5:
        // within noise or slower)
        constexpr bool PF2 = LT::HGLOBAL;
        double2v an2 = an, bn2 = bn, wm0 = wn0, wm1 = wn1;
        if constexpr (PF2) {
            const int k1 = k0 + 1 < Hb ? k0 + 1 : k0;
            an2 = ld2(ga + 2 * (k1 - l0));
            bn2 = ld2(gb + 2 * (k1 - m0));
            wm0 = ld2(W + 4 * k1 * nb);
            wm1 = ld2(W + 4 * k1 * nb + 2);
        }
        auto trip = [&](const double2v& anew, const double2v& bnew, const double2v& w0,
                        const double2v& w1) {
#pragma unroll
            for (int i = TS - 1; i > 0; --i) {
                av[i] = av[i - 1];
                bv[i] = bv[i - 1];
            }
            av[0] = anew;
            bv[0] = bnew;
            double px[TS], py[TS];   // W~ g_b for every column
#pragma unroll
            for (int j = 0; j < TS; ++j) {
                px[j] = w0.x * bv[j].x + w0.y * bv[j].y;
                py[j] = w1.x * bv[j].x + w1.y * bv[j].y;
            }
            // two FMAs per entry (c + a_x px) + a_y py: 2 TS^2 + 4 TS operations per trip
            // instead of 3 TS^2 + 4 TS for c + (a_x px + a_y py) (round 5: c2 +1.4 %)
#pragma unroll
            for (int i = 0; i < TS; ++i)
#pragma unroll
                for (int j = 0; j < TS; ++j) c[i][j] = fma(av[i].y, py[j], fma(av[i].x, px[j], c[i][j]));
        };
        // one operand set loaded a step ahead (two on the workspace plans).  The round-5
        // ping-pong form for the LDS factors (two operand sets held ahead of the other
        // trip's arithmetic) saved 3k cycles per IPM iteration at B = 1 and nothing at
        // B = 1024 (profiles/r05_ab_pingpong.txt), for 88 B more stack per lane and
        // +42 % HBM bytes on c2; round 6 returned to this loop (verdict r05 item 3)
        for (int k = k0; k < Hb; ++k) {
            const double2v acur = an, bcur = bn, w0 = wn0, w1 = wn1;
            if constexpr (PF2) {
                an = an2;
                bn = bn2;
                wn0 = wm0;
                wn1 = wm1;
                const int kn = k + 2 < Hb ? k + 2 : Hb - 1;
                an2 = ld2(ga + 2 * (kn - l0));
                bn2 = ld2(gb + 2 * (kn - m0));
                wm0 = ld2(W + 4 * kn * nb);
                wm1 = ld2(W + 4 * kn * nb + 2);
            } else {
                const int kn = k + 1 < Hb ? k + 1 : k;   // the last step reloads its own
                an = ld2(ga + 2 * (kn - l0));
                bn = ld2(gb + 2 * (kn - m0));
                wn0 = ld2(W + 4 * kn * nb);
                wn1 = ld2(W + 4 * kn * nb + 2);
            }
            trip(acur, bcur, w0, w1);
        }
#pragma unroll
        for (int di = 0; di < TS; ++di)
#pragma unroll
            for (int dj = 0; dj < TS; ++dj) {
                const int l = l0 + di, lp = m0 + dj;
                if (l >= Hb || lp >= Hb || (a_ == b_ && lp > l)) continue;
                const int row = a_ * Hb + l, col = b_ * Hb + lp;
                double acc = c[di][dj];
                if (row == col) acc += 2.0 * u2 * P.R[a_] + d[L.m + row] + d[L.m + N + row] + rho;
                L.H[roff(row) + col] = acc;
            }
    }
}

template <class LT, class PD>
__device__ void assemble(const cParams& P, const LT& L, PD d, double rho) {
    const int tid = threadIdx.x, V = L.V, Hb = L.Hb, nb = L.nb;
    const double u2 = P.uLim * P.uLim;
    // phase 1: W~ blocks [k][a>=b] (2x2) and the omega-coupling vector in y-space (yb)
    const int nW = Hb * nb;
    PROF_T0_FINE();
    for (int e = tid; e < nW + V * Hb; e += NT) {
        if (e < nW) {
            const int k = e / nb, ab = e % nb;
            int a_ = 0;
            while ((a_ + 1) * (a_ + 2) / 2 <= ab) ++a_;
            const int b_ = ab - a_ * (a_ + 1) / 2;
            double w00 = 0.0, w01 = 0.0, w11 = 0.0;
            if (a_ == b_) {
                const double qk = 2.0 * u2 * ((k == Hb - 1) ? P.Qf[a_] : P.Q[a_]);
                w00 = qk;
                w11 = qk;
                for (int wv = 0; wv < V; ++wv) {
                    if (wv == a_) continue;
                    const int i = a_ < wv ? a_ : wv, j = a_ < wv ? wv : a_;
                    const int r = pair_index(i, j, V) * Hb + k;
                    const double e0 = L.rowE[2 * r], e1 = L.rowE[2 * r + 1], dr = d[r];
                    w00 += dr * e0 * e0;
                    w01 += dr * e0 * e1;
                    w11 += dr * e1 * e1;
                }
                for (int o = 0; o < L.O; ++o) {
                    const int r = L.mp + (a_ * L.O + o) * Hb + k;
                    const double e0 = L.rowE[2 * r], e1 = L.rowE[2 * r + 1], dr = d[r];
                    w00 += dr * e0 * e0;
                    w01 += dr * e0 * e1;
                    w11 += dr * e1 * e1;
                }
            } else {
                const int r = pair_index(b_, a_, V) * Hb + k;   // b_ < a_
                const double e0 = L.rowE[2 * r], e1 = L.rowE[2 * r + 1], dr = -d[r];
                w00 = dr * e0 * e0;
                w01 = dr * e0 * e1;
                w11 = dr * e1 * e1;
            }
            auto* W = L.Wt + 4 * e;
            W[0] = w00; W[1] = w01; W[2] = w01; W[3] = w11;
        } else {
            const int q = e - nW, v = q / Hb, k = q % Hb;
            double s0, s1;
            incident_sum(L, v, k, [&](int r) { return d[r] * L.rowW[r]; }, s0, s1);
            L.yb[2 * q] = s0;
            L.yb[2 * q + 1] = s1;
        }
    }
    double ww = 0.0;
    for (int r = tid; r < L.m; r += NT) ww += d[r] * L.rowW[r] * L.rowW[r];
    double red[4] = {ww, 0.0, 0.0, 0.0};
    // buffer 2: the IPM's assembly follows the residuals' second reduction (buffer 1)
    // and the polish's follows ph_polish_accept's second (buffer 0), both with no
    // barrier between them (the round-5 buffer 1 raced with the residuals')
    block_reduce4<1, 2>(red, 0, L.red);
    PROF_ACC_FINE0(25);
    // phase 2: K_uu lower triangle in TS x TS tiles (assemble_tiles); 4 x 4 where
    // there are enough of them to give every thread two (only the workspace plans
    // have such horizons: the LDS-plan kernels do not carry the 4 x 4 registers)
    const int T4 = (Hb + 3) >> 2, PV = V * (V - 1) / 2;
    // LDS factors (c2, c5) take the 4 x 4 tiles too since round 5: at c2 the 210 tiles
    // leave 46 of 256 threads idle, but each trip serves 16 entries for the same four
    // loads, and the busiest thread does 20 trips instead of 32 (c2 +0.6 %, c4 +1.9 %,
    // scratch 196 -> 236 B per lane)
    if constexpr (LT::HGLOBAL) {
        if (V * (T4 * (T4 + 1) / 2) + PV * T4 * T4 >= 2 * NT) assemble_tiles<4>(P, L, d, rho);
        else assemble_tiles<2>(P, L, d, rho);
    } else {
        (void)T4;
        (void)PV;
        assemble_tiles<4>(P, L, d, rho);
#ifdef SCPQP_DIAG_X2_ASM   // counter attribution: the tiles again (the same values stored)
        assemble_tiles<4>(P, L, d, rho);
#endif
    }
    PROF_ACC_FINE0(26);
    const int N = L.N;
    toeplitz_t_apply(L, L.yb, [&](int e, double tt) { L.H[roff(N) + e] = tt; });
    if (tid == 0) L.H[roff(N) + N] = red[0] + d[L.mc - 1] + rho;
    bar();
    PROF_ACC_FINE0(27);
}

// ---------------------------------------------------------------------------
// Factorisation  K = L D L'  (L unit lower, stored strictly below the
// diagonal of H; dinv = 1/D), blocked right-looking, panel width CB, with a
// one-panel look-ahead.  Per panel step (one barrier):
//   * wave 0 applies the current panel's rank-CB update to the NEXT panel's
//     columns and factors that panel in registers (pivots and panel-row
//     entries broadcast with v_readlane: no barrier inside the panel);
//   * waves 1.. apply the current panel's update to the columns beyond the
//     next panel, H_ik -= sum_c L_ic D_c L_kc, in 2x2 register tiles with
//     16-byte loads.
// The serial panel chain of wave 0 thus runs concurrently with the trailing
// update instead of between two barriers.  Pivots and the failure flag are
// double-buffered by panel parity.  Returns false on a non-positive pivot
// (K not numerically positive definite).
// Contract: after the factorisation the strictly lower entries of H hold L (unit
// lower, diagonal implicit) and dinv holds 1/D.  The diagonal slots of H are
// unspecified: most hold D (1/D) rounded, and the last row's holds its updated K
// entry when the last panel is the omega row alone (n = 8 k + 1, panel_factor's
// jb == 1 path).  No reader uses them.
// ---------------------------------------------------------------------------
#define CB 8   // panel width (4 measured slower: DESIGN §3)

// 1/x for a positive finite pivot: v_rcp_f64 + two Newton steps (full precision,
// a fraction of the IEEE division sequence's latency on the serial panel path).
__device__ __forceinline__ double recip(double x) {
    double r = __builtin_amdgcn_rcp(x);
    double e = fma(-x, r, 1.0);
    r = fma(r, e, r);
    e = fma(-x, r, 1.0);
    return fma(r, e, r);
}

__device__ __forceinline__ bool wave0() {
    return __builtin_amdgcn_readfirstlane(threadIdx.x) < 64;   // wave-uniform branch
}
// The serial parts of a problem (panel factorisation, triangular solves) run on
// one wave, the lead.  Each workgroup picks its lead on a different SIMD from
// the other workgroups resident on its CU (lead_wave_elect), so their serial
// chains do not share an issue port.
__device__ __forceinline__ int wave_id() {
    return __builtin_amdgcn_readfirstlane(threadIdx.x) >> 6;
}
__device__ __forceinline__ bool is_lead(int lead) { return wave_id() == lead; }
// The lead's serial chains (panel factorisation, triangular solves) are the problem's
// critical path; the other waves on its SIMD belong to other problems.  Raise the lead's
// issue priority over them for the chain's duration (s_setprio; MI355X_MICROARCH.md,
// "Two waves per SIMD": priority outranks age).
// c2 84.7k -> 88.3k, c4 145k -> 149k solves/s (profiles/r03_ab_prio.txt).  Giving the
// whole workgroup of a long-running problem priority instead (an age rule) changed nothing.
__device__ __forceinline__ void lead_prio_up() { __builtin_amdgcn_s_setprio(2); }
__device__ __forceinline__ void lead_prio_down() { __builtin_amdgcn_s_setprio(0); }

// Panel factorisation (the lead wave): the panel of columns [r0, r0 + jb) in registers,
// rows i = r0 + lane + 64 t.  If jp >= 0 the panel first receives the rank-CB update of
// the previous panel(s) (columns [jp, jp + nprev CB), pivots dprev).  Branch-free: rows
// >= n read a clamped row, columns >= jb of the last panel are padded with an identity
// block (D = 1, no coupling), and entries above the diagonal (lane < c) only hold values
// that are never broadcast or stored.  Round-3 form; its chain is shorter than the
// column-by-column form's (two v_readlane round trips per pivot column):
//  * look-ahead from the most recent panel: its D-scaled rows r0 .. r0 + 7 were left in
//    LDS (ldbuf, 8 x 8) by the previous step's lead, so they are read as broadcast
//    loads instead of 64 v_readlane pairs; an older panel (grouped trailing update)
//    still takes the readlane path;
//  * the 8 x 8 diagonal block is gathered to every lane at once (36 independent
//    readlanes) and factored on uniform values (L D L', right-looking), so the chain
//    per column is the reciprocal and two FMAs instead of two readlane round trips;
//  * every row then applies the block's factor by forward substitution
//    (p_ic -= (p_ic' / D_c') U_cc', U = L D unscaled), which for the block's own rows
//    repeats the uniform factorisation operation for operation.
template <int RS, bool OPQ, class HP>
__device__ __forceinline__ void panel_factor(HP H, ldouble* dinv, int n, int r0, int jb, int jp,
                                              const ldouble* dprev, ldouble* dout, lint* flag,
                                              int nprev, ldouble* ldbuf) {
    // OPQ (kernels with more than two row slots, c3): the lane index through an empty
    // volatile asm, so that the values derived from it (the identity padding, the look-ahead
    // row addresses) are formed per panel step instead of being hoisted out of the step loop,
    // where at RMAX = 4 they were spilled to scratch and reloaded on the lead's chain every
    // step (c3 +4.5 %; at RMAX = 2 nothing is spilled and the recomputation costs c2 3 %:
    // profiles/r06_ab_panel_lane.txt)
    int lane = threadIdx.x & 63;
    if constexpr (OPQ) asm volatile("" : "+v"(lane));
    PROF_T0_FINE();
    double p[RS][CB];
    int ro[RS];
#pragma unroll
    for (int t = 0; t < RS; ++t) {
        const int i = r0 + lane + 64 * t;
        ro[t] = roff(i < n ? i : n - 1);
#pragma unroll
        for (int c = 0; c < CB; c += 2) {
            const double2v v = ld2(H + ro[t] + r0 + c);
            p[t][c] = v.x;
            p[t][c + 1] = v.y;
        }
    }
#ifdef SCPQP_PROF_FINE
    __builtin_amdgcn_s_waitcnt(0);
#endif
    PROF_ACC_FINE(18);
    for (int q = 0; jp >= 0 && q < nprev; ++q) {
        double li[RS][CB];
#pragma unroll
        for (int t = 0; t < RS; ++t)
#pragma unroll
            for (int c = 0; c < CB; c += 2) {
                const double2v v = ld2(H + ro[t] + jp + q * CB + c);
                li[t][c] = v.x;
                li[t][c + 1] = v.y;
            }
        if (q == nprev - 1) {
            // the previous step's D-scaled rows r0 + c, two columns per round
#pragma unroll
            for (int c = 0; c < CB; c += 2) {
                double lk0[CB], lk1[CB];
#pragma unroll
                for (int c2 = 0; c2 < CB; c2 += 2) {
                    const double2v v0 = ld2(ldbuf + c * CB + c2), v1 = ld2(ldbuf + (c + 1) * CB + c2);
                    lk0[c2] = v0.x; lk0[c2 + 1] = v0.y;
                    lk1[c2] = v1.x; lk1[c2 + 1] = v1.y;
                }
#pragma unroll
                for (int t = 0; t < RS; ++t) {
                    double s0 = li[t][0] * lk0[0], s1 = li[t][0] * lk1[0];
#pragma unroll
                    for (int c2 = 1; c2 < CB; ++c2) {
                        s0 = fma(li[t][c2], lk0[c2], s0);
                        s1 = fma(li[t][c2], lk1[c2], s1);
                    }
                    p[t][c] -= s0;
                    p[t][c + 1] -= s1;
                }
            }
        } else {
            double ld[CB];
#pragma unroll
            for (int c = 0; c < CB; ++c) ld[c] = li[0][c] * dprev[q * CB + c];
#pragma unroll
            for (int c = 0; c < CB; ++c) {
                double lk[CB];
#pragma unroll
                for (int c2 = 0; c2 < CB; ++c2) lk[c2] = readlane_d(ld[c2], c);
#pragma unroll
                for (int t = 0; t < RS; ++t) {
                    double sacc = 0.0;
#pragma unroll
                    for (int c2 = 0; c2 < CB; c2 += 2) sacc += li[t][c2] * lk[c2] + li[t][c2 + 1] * lk[c2 + 1];
                    p[t][c] -= sacc;
                }
            }
        }
    }
#pragma unroll
    for (int t = 0; t < RS; ++t) {
        const int i = r0 + lane + 64 * t;
#pragma unroll
        for (int c = 0; c < CB; ++c)
            p[t][c] = (i < n && c < jb) ? p[t][c] : ((t == 0 && lane == c) ? 1.0 : 0.0);
    }
    PROF_ACC_FINE(19);
    if (jb == 1) {
        // the last panel of n = 8 k + 1 (every shape with V Hb a multiple of 8: the omega
        // row alone): its pivot is the updated diagonal entry.  Nothing of this panel is
        // read later but dinv (no trailing columns, no look-ahead rows, the diagonal of L
        // is implicit), so the 8 x 8 block factorisation, the row substitution and the
        // stores are skipped; D and 1/D are the values they would produce.
        const double D = readlane_d(p[0][0], 0);
        if (lane == 0) {
            dinv[r0] = recip(D);
            dout[0] = D;
            flag[0] = !(D > 0.0) || !isfinite(D);
        }
        return;
    }
    double inv[CB], dg[CB];
    int bad = 0;
    double u0[CB];   // slot 0's unscaled entries (the next step's look-ahead rows)
    // Two columns per round (round 6).  Column c's entries U0 (rows c..7) and column
    // c + 1's, not yet updated by column c (V, rows c + 1..7), are broadcast with one round
    // of v_readlane; the pair's pivots come from the 2 x 2 block [d0 b; b e]: d1 = det / d0
    // with det = d0 e - b^2, so 1/d0 and 1/det are computed side by side and 1/d1 = d0 / det,
    // instead of 1/d1 after 1/d0 and a second readlane round (the round-5 column-by-column
    // chain).  Column c + 1 of the block rows, updated by column c (W), is formed on
    // uniform values with the column-by-column form's own operations, so every entry but
    // the second pivot of a pair is computed as before.
#pragma unroll
    for (int c = 0; c < CB; c += 2) {
        double U0[CB], V[CB], W[CB];
#pragma unroll
        for (int c2 = c; c2 < CB; ++c2) U0[c2] = readlane_d(p[0][c], c2);
#pragma unroll
        for (int c2 = c + 1; c2 < CB; ++c2) V[c2] = readlane_d(p[0][c + 1], c2);
        const double d0 = U0[c], b = U0[c + 1], e = V[c + 1];
        const double det = fma(d0, e, -(b * b));
        const double i0 = recip(d0), rdet = recip(det);
        const double i1 = d0 * rdet;
        dg[c] = d0;
        dg[c + 1] = det * i0;
        bad |= !(d0 > 0.0) || !isfinite(d0) || !(det > 0.0) || !isfinite(det);
        inv[c] = i0;
        inv[c + 1] = i1;
#pragma unroll
        for (int c2 = c + 2; c2 < CB; ++c2) W[c2] = fma(-(U0[c2] * i0), b, V[c2]);
        u0[c] = p[0][c];
#pragma unroll
        for (int t = 0; t < RS; ++t) {
            const double l0 = p[t][c] * i0;
            const double pc1 = fma(-l0, b, p[t][c + 1]);
            if (t == 0) u0[c + 1] = pc1;
            const double l1 = pc1 * i1;
#pragma unroll
            for (int c2 = c + 2; c2 < CB; ++c2) p[t][c2] = fma(-l1, W[c2], fma(-l0, U0[c2], p[t][c2]));
            p[t][c] = l0;
            p[t][c + 1] = l1;
        }
    }
    if (lane < CB && lane < jb) {
        double iv = inv[0], dv = dg[0];
#pragma unroll
        for (int c = 1; c < CB; ++c) {
            iv = lane == c ? inv[c] : iv;
            dv = lane == c ? dg[c] : dv;
        }
        dinv[r0 + lane] = iv;
        dout[lane] = dv;
    }
    PROF_ACC_FINE(20);
#pragma unroll
    for (int t = 0; t < RS; ++t) {
        const int i = r0 + lane + 64 * t;
        if (i < n) {
#pragma unroll
            for (int c = 0; c < CB; c += 2)
                if (c < jb && c <= lane + 64 * t) st2(H + ro[t] + r0 + c, double2v{p[t][c], p[t][c + 1]});
        }
    }
    // rows r0 + 8 .. r0 + 15 (the next panel's diagonal-block rows), D-scaled, for the
    // next step's look-ahead; the lead alone reads them, so no barrier is needed
    if (lane >= CB && lane < 2 * CB) {
#pragma unroll
        for (int c = 0; c < CB; c += 2) st2(ldbuf + (lane - CB) * CB + c, double2v{u0[c], u0[c + 1]});
    }
    if (lane == 0) flag[0] = bad;
    PROF_ACC_FINE(21);
}

// Rank-CB update of panel j0 (pivots dcur) on rows/columns >= r1, by threads
// [t0, t0 + nth) of the workgroup.  2x2 tiles (ti >= tk) enumerated linearly
// so every thread gets ceil(ntile / nth) tiles; two tiles per pass so their
// LDS latencies overlap.  r1 is even, so the (i0, i0 + 1) element of a
// diagonal tile is row i0's padding slot, and row n (i1 == n) is the spare
// row the plan allocates: the tile stores need no predicates.
// NEUTRAL (diagnostic builds only, SCPQP_DIAG_X2_TRAIL): the same loads and stores with the
// entries unchanged, so that a second pass attributes the update's LDS bank conflicts
template <class HP, bool NEUTRAL = false>
__device__ __forceinline__ void trailing_update(HP H, int n, int j0, int r1, const ldouble* dcur,
                                                int t0, int nth) {
    double dc[CB];
#pragma unroll
    for (int c = 0; c < CB; ++c) dc[c] = dcur[c];
    const int T = (n - r1 + 1) >> 1;
    const int ntile = T * (T + 1) / 2;
    for (int t = t0; t < ntile; t += 2 * nth) {
        const int tb = t + nth < ntile ? t + nth : t;
        int ia[2], ka[2];
        tri_decode(t, ia[0], ka[0]);
        tri_decode(tb, ia[1], ka[1]);
        double sm[2][4];
#pragma unroll
        for (int u2 = 0; u2 < 2; ++u2) {
            const int o0 = roff(r1 + 2 * ia[u2]), o1 = roff(r1 + 2 * ia[u2] + 1);
            const int q0 = roff(r1 + 2 * ka[u2]), q1 = roff(r1 + 2 * ka[u2] + 1);
            double s00 = 0.0, s01 = 0.0, s10 = 0.0, s11 = 0.0;
#pragma unroll
            for (int c = 0; c < CB; c += 2) {
                const double2v x0 = ld2(H + o0 + j0 + c), x1 = ld2(H + o1 + j0 + c);
                const double2v y0 = ld2(H + q0 + j0 + c), y1 = ld2(H + q1 + j0 + c);
                const double e0 = x0.x * dc[c], e1 = x0.y * dc[c + 1];
                const double f0 = x1.x * dc[c], f1 = x1.y * dc[c + 1];
                // two FMAs per column pair ((s + e0 y.x) + e1 y.y, round 5: c2 +0.2 %,
                // c4 +0.5 % over s + (e0 y.x + e1 y.y))
                s00 = fma(e1, y0.y, fma(e0, y0.x, s00));
                s01 = fma(e1, y1.y, fma(e0, y1.x, s01));
                s10 = fma(f1, y0.y, fma(f0, y0.x, s10));
                s11 = fma(f1, y1.y, fma(f0, y1.x, s11));
            }
            sm[u2][0] = s00; sm[u2][1] = s01; sm[u2][2] = s10; sm[u2][3] = s11;
        }
#pragma unroll
        for (int u2 = 0; u2 < 2; ++u2) {
            if (u2 == 1 && tb == t) break;
            const int i0 = r1 + 2 * ia[u2], k0 = r1 + 2 * ka[u2];
            const int o0 = roff(i0), o1 = roff(i0 + 1);
            const double f = NEUTRAL ? 0.0 : 1.0;
            H[o0 + k0] -= f * sm[u2][0];
            H[o0 + k0 + 1] -= f * sm[u2][1];
            H[o1 + k0] -= f * sm[u2][2];
            H[o1 + k0 + 1] -= f * sm[u2][3];
        }
    }
}

// The same rank-CB trailing update on the matrix cores, for a factor that lives in
// the global workspace (plan 2: 8 vehicles at Hp 30, n = 241).  There the VALU
// update is the factorisation's critical path (the lead wave waits ~95 % of each
// panel step at the barrier, profiles/r02_phases_fine.txt): 2 x 2 register tiles
// re-read their operands from L2 for every 4 outputs.  Here a wave takes whole
// 16 x 16 tiles (i >= k): K_ik -= sum_c (L_ic D_c) L_kc is two
// v_mfma_f64_16x16x4_f64 (CB = 8 = 2 x 4) with the old tile as the accumulator
// and the A operand negated, so the tile is loaded once and stored once.  KS
// 16x16x4 MFMAs per tile: the update's rank is 4 KS (CB, or 2 CB when paired).
// Operand layouts (gfx950): A[row = lane & 15][k = lane >> 4], B[k = lane >> 4]
// [col = lane & 15], C/D col = lane & 15, row = (lane >> 4) + 4 r.  Entries above
// the diagonal of a diagonal tile and outside the matrix are neither read nor
// written (packed rows end at the diagonal).
typedef double double4v __attribute__((ext_vector_type(4)));

// U tiles are in flight per wave so that their L2 loads overlap (round 2, two panels per
// update: 4 at a 256-VGPR budget, c3 2.37k -> 2.73k solves/s; round 5, four panels: 2).
// part: 0 all tiles; 1 .. np the tile columns between the cuts that split the tile
// count into np equal shares (column tile 0, the next panels' columns, always in part 1).
// Tiles are enumerated column by column, so each part is a contiguous range.
template <int U, int KS, class HP>
__device__ __forceinline__ void trailing_update_mfma(HP H, int n, int j0, int r1, const ldouble* dcur,
                                                     int wave, int nwave, int part = 0, int np = 1) {
    const int lane = threadIdx.x & 63, lr = lane & 15, lk = lane >> 4;
    double dk[KS];
#pragma unroll
    for (int kk = 0; kk < KS; ++kk) dk[kk] = dcur[4 * kk + lk];
    const int T = (n - r1 + 15) >> 4;
    const int ntile = T * (T + 1) / 2;
    int tb = 0, te = ntile;
    if (part != 0) {
        // part p of np: the tile columns from the (p-1)-th to the p-th cut, the k-th cut
        // being the first tile-column boundary with >= k ntile / np tiles before it
        // (tile column 0 always in part 1)
        int js = 1, cum = T;   // tiles in the tile columns < js
        for (int k = 1; k < np; ++k) {
            while (js < T && np * cum < k * ntile) {
                cum += T - js;
                ++js;
            }
            if (k == part - 1) tb = cum;
            if (k == part) te = cum;
        }
    }
    for (int t = tb + wave; t < te; t += U * nwave) {
        double a[U][KS], b[U][KS];
        double4v acc[U];
        int oc[U][4];
        bool ok[U][4];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int tu = t + u * nwave;
            const bool live = tu < te;
            int I = 0, J = 0;   // column-major order: the reversed row-major decode, mirrored
            tri_decode(ntile - 1 - (live ? tu : t), J, I);
            I = T - 1 - I;
            J = T - 1 - J;
            const int i0 = r1 + 16 * I, k0 = r1 + 16 * J;
            const int ia = min(i0 + lr, n - 1), kb = min(k0 + lr, n - 1);
            const int oa = roff(ia) + j0, ob = roff(kb) + j0;
#pragma unroll
            for (int kk = 0; kk < KS; ++kk) {
                a[u][kk] = -H[oa + 4 * kk + lk] * dk[kk];
                b[u][kk] = H[ob + 4 * kk + lk];
            }
            const int kc = k0 + lr;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int ci = i0 + lk + 4 * r;
                ok[u][r] = live && ci < n && kc <= ci;
                oc[u][r] = roff(ok[u][r] ? ci : 0) + (ok[u][r] ? kc : 0);
                acc[u][r] = ok[u][r] ? (double)H[oc[u][r]] : 0.0;
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
#pragma unroll
            for (int kk = 0; kk < KS; ++kk)
                acc[u] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[u][kk], b[u][kk], acc[u], 0, 0, 0);
        }
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
            for (int r = 0; r < 4; ++r)
                if (ok[u][r]) H[oc[u][r]] = acc[u][r];
    }
}

// Grouped trailing update (factor in the global workspace): the update streams
// the whole remaining factor through L2 once per application, and for n = 241 it
// is the factorisation's critical path.  The trailing waves therefore apply the
// rank-(G CB) update of G panels at once, spread over the next group's G steps
// (trailing_update_mfma parts); the lead's look-ahead covers every panel factored
// since the last group update.  1/G of the passes over the factor (G = 2: c3
// 3.51-3.55k -> 4.04-4.07k solves/s).
// panels per grouped trailing update: 4 since round 5 (c3 +1-2 % against 2 in one session,
// HBM traffic 2.93 -> 2.35 TB per launch; unsplit in round 2 it measured slower)
constexpr int kGroup = 4;
static_assert(kPivSlot + 2 * kGroup * CB == red_size(true) && kPivSlot + 2 * CB == red_size(false),
              "the pivot buffer of red_size");

template <class LT>
__device__ bool cholesky(const LT& L) {
    const int n = __builtin_amdgcn_readfirstlane(L.n);
    constexpr int RS = LT::RMAX;   // row slots per lane in the panel
    constexpr int G = LT::HGLOBAL ? kGroup : 1;
    lint* flag = (lint*)(L.red + kRedFlag);   // [step parity]
    ldouble* ldbuf = L.red;              // [CB][CB] look-ahead rows (panel_factor; red is idle here)
    ldouble* dbuf = L.red + kPivSlot;    // pivots [step mod 2G][CB]; a group's slots are adjacent
    PROF_T0();
    for (int r0 = 0, s = 0; r0 < n; r0 += CB, ++s) {
        const int par = s & 1;
        const int jb = min(CB, n - r0), r1 = r0 + jb;
        // look-ahead source: the panels factored since the last group update
        const int sg = s % G;
        const int np = G == 1 ? 1 : (sg == 0 ? G : sg);
        const int jp = r0 - np * CB;   // < 0 at the first step: no look-ahead
        // (s - np) & (2G - 1): a valid slot also at s < np (2G is a power of two), where
        // jp < 0 and the pointer is not dereferenced
        const ldouble* dprev = dbuf + ((s - np) & (2 * G - 1)) * CB;
        if (is_lead(L.lead)) {
            // rows r0 .. n-1 only: once they fit one slot per lane the panel
            // runs with one register row (half the VALU work of the chain)
            ldouble* dn = dbuf + (s % (2 * G)) * CB;
            lead_prio_up();
            constexpr bool OPQ = RS > 2;
            if (RS == 1 || n - r0 <= 64) panel_factor<1, OPQ>(L.H, L.dinv, n, r0, jb, jp, dprev, dn, flag + par, np, ldbuf);
            else panel_factor<RS, OPQ>(L.H, L.dinv, n, r0, jb, jp, dprev, dn, flag + par, np, ldbuf);
            lead_prio_down();
        } else if (jp >= 0 || (G > 1 && s >= G)) {
            const int tw = (wave_id() - L.lead + NWAVE - 1) % NWAVE;   // 0 .. NWAVE-2
            if constexpr (LT::HGLOBAL) {
                // tiles in flight per wave: 2 (round 5, with the group of four's eight MFMAs
                // per tile: c3 5.92-6.07k -> 6.39-6.44k against 4, 1 within noise of 2;
                // profiles/r05_ab_mfma_tiles.txt)
                constexpr int U = 2;
                // the previous group's update in G parts, part sg + 1 on step sg of this
                // group: the left tile columns (they hold the next panels) on its first
                // step, so every later step's panel chain runs beside a share of the update
                const int s0 = s - sg;   // this group's first step
                if (s0 >= G)
                    trailing_update_mfma<U, G * CB / 4>(L.H, n, (s0 - G) * CB, s0 * CB + CB,
                                                        dbuf + ((s0 - G) & (2 * G - 1)) * CB,
                                                        tw, NWAVE - 1, sg + 1, G);
            } else {
                trailing_update(L.H, n, jp, r1, dprev, tw * 64 + (int)(threadIdx.x & 63), NT - 64);
#ifdef SCPQP_DIAG_X2_TRAIL   // counter attribution: a result-neutral second pass
                trailing_update<decltype(L.H), true>(L.H, n, jp, r1, dprev, tw * 64 + (int)(threadIdx.x & 63), NT - 64);
#endif
            }
        }
#if defined(SCPQP_PROF) && defined(SCPQP_PROF_FINE)
        unsigned long long _pb = __builtin_amdgcn_s_memtime();
#endif
        bar();
#if defined(SCPQP_PROF) && defined(SCPQP_PROF_FINE)
        // barrier waits of the lead wave (panel chain) and of one trailing-update wave
        if (threadIdx.x == 64 * L.lead) atomicAdd(&g_prof[22], __builtin_amdgcn_s_memtime() - _pb);
        if (threadIdx.x == 64 * ((L.lead + 1) & 3)) atomicAdd(&g_prof[23], __builtin_amdgcn_s_memtime() - _pb);
#endif
        if (flag[par]) return false;
    }
    PROF_ACC(13);
    return true;
}

// ---------------------------------------------------------------------------
// Solve K x = b with K = L D L'.  The lead wave only; rows i = lane + 64 t (t < R).
// Unit-lower forward / backward substitution: the dependency chain per step
// is one v_readlane broadcast of the owner lane's value plus one FMA.  L is
// streamed 4 columns (forward) / 4 rows (backward) at a time into registers,
// double-buffered, so the LDS latency hides behind the dependent steps.
// (Measured alternatives, tools/probe/solve_probe.hip and DESIGN §3: ping-pong
// buffers with bounds-free full chunks, v_writelane capture, and a blocked
// variant that solves 8 x 8 diagonal blocks on uniform values; the first two
// are faster in isolation but slower inside the kernel, the third is slower.)
// ---------------------------------------------------------------------------

constexpr int kSolveChunk = 4;    // chunk of a factor in LDS
constexpr int kSolveChunkG = 8;   // chunk of a factor in the workspace: twice the steps cover the L2 latency
template <int R, class HP, int SCH, bool RTN = false>
struct Solver {   // SCH: chunk (columns / rows) streamed per step group; RTN: n not a
                  // compile-time constant (the chunk loops stay rolled, below)
    static_assert(SCH % 2 == 0 && 64 % SCH == 0, "chunks tile the 64-row slots");
    HP H;                   // factor (LDS or workspace)
    const ldouble* dinv;
    int lane, n, ld;
    double r[R], xf[R];
    int ii[R], ro[R], ic[R];
    double cur[R][SCH], nxt[R][SCH];

    // No per-lane predicates in the step loops: rows of a lane that is already
    // final (i <= j in the forward sweep, i >= j backward) read entries past
    // their row end and accumulate garbage, so every final value is captured
    // into xf at the step that produces it.  Rows >= n read a clamped row.
    __device__ __forceinline__ Solver(HP H_, const ldouble* dinv_, int n_, int ld_,
                                      const ldouble* bvec)
        : H(H_), dinv(dinv_), n(n_), ld(ld_) {
        lane = threadIdx.x & 63;
#pragma unroll
        for (int t = 0; t < R; ++t) {
            ii[t] = lane + 64 * t;
            ic[t] = ii[t] < n ? ii[t] : n - 1;
            ro[t] = roff(ic[t]);
            r[t] = ii[t] < n ? bvec[ii[t]] : 0.0;
            xf[t] = 0.0;
        }
    }
    __device__ __forceinline__ void load_cols(double (&dst)[R][SCH], int jc) {
#pragma unroll
        for (int t = 0; t < R; ++t)
#pragma unroll
            for (int q = 0; q < SCH; q += 2) {
                const double2v v = ld2(H + ro[t] + jc + q);
                dst[t][q] = v.x;
                dst[t][q + 1] = v.y;
            }
    }
    __device__ __forceinline__ void load_rows(double (&dst)[R][SCH], int jc) {
#pragma unroll
        for (int q = 0; q < SCH; ++q) {
            const int row = jc + q < n ? jc + q : n - 1;
#pragma unroll
            for (int t = 0; t < R; ++t) dst[t][q] = H[roff(row) + ic[t]];
        }
    }
    __device__ __forceinline__ void shift() {
#pragma unroll
        for (int t = 0; t < R; ++t)
#pragma unroll
            for (int q = 0; q < SCH; ++q) cur[t][q] = nxt[t][q];
    }
    // the solution entry j (uniform xj) into its owner lane (v_writelane through M0 is
    // bitwise the same but kept the sweep from unrolling: solves 21.2k -> 31.3k cycles per
    // IPM iteration at B = 1, c2 -7 %, profiles/r05_ab_writelane.txt)
    __device__ __forceinline__ double capture(double xj, int j, double old) const {
        return (lane == (j & 63)) ? xj : old;
    }
    // forward over the columns owned by slot T (compile-time owner); slots < T are final
    template <int T>
    __device__ __forceinline__ void fwd() {
        if constexpr (T < R) {
            const int jend = min(n, 64 * (T + 1));
            auto chunk = [&](int jc) {
                if (jc + SCH < n) load_cols(nxt, jc + SCH);
#pragma unroll
                for (int q = 0; q < SCH; ++q) {
                    const int j = jc + q;
                    if (j < jend) {
                        const double xj = readlane_d(r[T], j & 63);
                        r[T] -= cur[T][q] * xj;
                        xf[T] = capture(xj, j, xf[T]);
#pragma unroll
                        for (int t = T + 1; t < R; ++t) r[t] -= cur[t][q] * xj;
                    }
                }
                shift();
            };
            if constexpr (RTN) {
                // with a run-time n the compiler unrolled this loop once per possible
                // remainder (248 VGPRs, stack reloads inside the sweep: c5's mixed
                // horizons); rolled it stays one chunk body
#pragma unroll 1
                for (int jc = 64 * T; jc < jend; jc += SCH) chunk(jc);
            } else {
                for (int jc = 64 * T; jc < jend; jc += SCH) chunk(jc);
            }
        }
    }
    // backward over the rows owned by slot T; slots > T are final
    template <int T>
    __device__ __forceinline__ void bwd(int jlast) {
        if constexpr (T < R) {
            const int jstart = (T == R - 1) ? jlast : 64 * T + 64 - SCH;
            auto chunk = [&](int jc) {
                if (jc > 0) load_rows(nxt, jc - SCH);
#pragma unroll
                for (int q = SCH - 1; q >= 0; --q) {
                    const int j = jc + q;
                    if (j < n) {
                        const double xj = readlane_d(r[T], j & 63);
                        // the owner slot first: it carries the next step's broadcast
                        r[T] -= cur[T][q] * xj;
                        xf[T] = capture(xj, j, xf[T]);
#pragma unroll
                        for (int t = 0; t < T; ++t) r[t] -= cur[t][q] * xj;
                    }
                }
                shift();
            };
            if constexpr (RTN) {
#pragma unroll 1
                for (int jc = jstart; jc >= 64 * T; jc -= SCH) chunk(jc);
            } else {
                for (int jc = jstart; jc >= 64 * T; jc -= SCH) chunk(jc);
            }
        }
    }
    __device__ __forceinline__ void run(ldouble* x) {
        PROF_T0();
        // forward  L y = b
        load_cols(cur, 0);
        fwd<0>(); fwd<1>(); fwd<2>(); fwd<3>();
        PROF_ACC(14);
        // z = D^{-1} y
#pragma unroll
        for (int t = 0; t < R; ++t) {
            r[t] = xf[t] * dinv[ic[t]];
            xf[t] = 0.0;
        }
        // backward  L' x = z
        const int jlast = ((n - 1) / SCH) * SCH;
        load_rows(cur, jlast);
        bwd<3>(jlast); bwd<2>(jlast); bwd<1>(jlast); bwd<0>(jlast);
#pragma unroll
        for (int t = 0; t < R; ++t)
            if (ii[t] < n) x[ii[t]] = xf[t];
        PROF_ACC(15);
    }
};

template <int R, bool RTN, class LT>
__device__ __forceinline__ void chol_solve_r(const LT& L, const ldouble* bvec, ldouble* x) {
    Solver<R, decltype(L.H), (LT::HGLOBAL ? kSolveChunkG : kSolveChunk), RTN> S(L.H, L.dinv, L.n, L.ld, bvec);
    S.run(x);
}

// SH: the problem shape.  A run-time horizon (shapes 0 and 2) keeps the sweeps' chunk
// loops rolled; c5's horizon classes run as shapes 4-6 with n compiled in (the kernel's
// QP dispatch), unrolled like c2's (c5 B = 1 Hp 30: solves 62.3k -> 33.2k cycles per IPM
// iteration, c5 117.7k -> 135k solves/s, profiles/r05_ab_c5_solve_classes.txt).
template <int SH, class LT>
__device__ void chol_solve(const LT& L, const ldouble* bvec, ldouble* x) {
    constexpr bool RTN = shape_c(SH).H == 0;
#ifdef SCPQP_DIAG_X2_SOLVE   // counter attribution: the solve twice (the same x)
    for (int rep = 0; rep < 2; ++rep)
#endif
    if (is_lead(L.lead)) {
        const int n = L.n;
        constexpr int RM = LT::RMAX;
        lead_prio_up();
        if (RM == 1 || n <= 64) chol_solve_r<1, RTN>(L, bvec, x);
        else if (RM == 2 || n <= 128) chol_solve_r<(RM >= 2 ? 2 : 1), RTN>(L, bvec, x);
        else if (RM == 3 || n <= 192) chol_solve_r<(RM >= 3 ? 3 : 1), RTN>(L, bvec, x);
        else chol_solve_r<RM, RTN>(L, bvec, x);
        lead_prio_down();
    }
    bar();
}

// ---------------------------------------------------------------------------
// QCQP evaluation (SCP_controller.py:215-265) of the unscaled control vector u
// (LDS, [V*Hb]).  Positions go to L.pb.  Obstacle rows follow quirk B.4 when
// flagged: evaluated (nVeh-1-v) times (sum) and never for the last vehicle.
// ---------------------------------------------------------------------------
struct EvalRes {
    double obj, maxv, sumv;
    int feasible;
};

template <class LT>
__device__ EvalRes evaluate_u(const cParams& P, const LT& L, const ldouble* u, double* cveh,
                              double* cobs) {
    const int tid = threadIdx.x, V = L.V, Hb = L.Hb, O = L.O;
    toeplitz_apply(L, u, L.pb);
    bar();
    for (int e = tid; e < V * Hb; e += NT) {
        L.pb[2 * e] += L.p0[2 * e];
        L.pb[2 * e + 1] += L.p0[2 * e + 1];
    }
    bar();
    double obj = 0.0, mx = 0.0, sm = 0.0, nviol = 0.0;
    for (int e = tid; e < V * Hb; e += NT) {
        const int v = e / Hb, k = e % Hb;
        const double qk = (k == Hb - 1) ? P.Qf[v] : P.Q[v];
        const double ex = L.pb[2 * e] - L.ref[2 * e], ey = L.pb[2 * e + 1] - L.ref[2 * e + 1];
        obj += qk * (ex * ex + ey * ey) + P.R[v] * u[e] * u[e];
    }
    const bool quirk = (P.flags & SCPQP_FLAG_OBST_QUIRK) != 0;
    for (int r = tid; r < L.m; r += NT) {
        int i, j, o, k;
        row_decode(L.rinfo[r], i, j, o, k);
        const ldouble* pi = L.pb + (i * Hb + k) * 2;
        double dx, dy, D2;
        if (j >= 0) {
            dx = pi[0] - L.pb[(j * Hb + k) * 2];
            dy = pi[1] - L.pb[(j * Hb + k) * 2 + 1];
            D2 = P.D2veh[i * SCPQP_MAX_VEH + j];
        } else {
            dx = pi[0] - L.ob[(o * Hb + k) * 2];
            dy = pi[1] - L.ob[(o * Hb + k) * 2 + 1];
            D2 = P.D2obs[i * SCPQP_MAX_OBST + o];
        }
        const double c = D2 - (dx * dx + dy * dy);
        int reps = 1;
        if (j < 0 && quirk) reps = V - 1 - i;
        if (cveh && j >= 0) {
            cveh[(i * V + j) * Hb + k] = c;
            cveh[(j * V + i) * Hb + k] = c;
        }
        if (cobs && j < 0 && reps > 0) cobs[(i * O + o) * Hb + k] = c;
        if (c > P.ctol && reps > 0) {
            mx = fmax(mx, c);
            sm += c * reps;
            nviol += 1.0;
        }
    }
    double red[4] = {obj, sm, nviol, mx};
    block_reduce4<4>(red, 8, L.red);
    EvalRes res;
    res.obj = red[0];
    res.sumv = red[1];
    res.feasible = red[2] == 0.0;
    res.maxv = red[3];
    return res;
}

// ---------------------------------------------------------------------------
// Constraint linearisation at u-bar = L.ub (SCP_controller.py:93-128 in the
// factored form of SURVEY A.5), scaled rows:
//   e_r = 2 d uLim / nrm,  w_r = -1/nrm,  h_r = b_r / nrm,
//   nrm = || [a_r uLim, -1] ||,  a_r = -2 d' calB_i,k (+ 2 d' calB_j,k)
// ---------------------------------------------------------------------------
template <class LT>
__device__ void linearise_rows(const cParams& P, const LT& L) {
    const int tid = threadIdx.x, Hb = L.Hb;
    toeplitz_apply(L, L.ub, L.ya);
    bar();
    for (int e = tid; e < L.V * Hb; e += NT) {
        L.pb[2 * e] = L.p0[2 * e] + L.ya[2 * e];
        L.pb[2 * e + 1] = L.p0[2 * e + 1] + L.ya[2 * e + 1];
    }
    bar();
    for (int r = tid; r < L.m; r += NT) {
        int i, j, o, k;
        row_decode(L.rinfo[r], i, j, o, k);
        const ldouble* pi = L.pb + (i * Hb + k) * 2;
        const ldouble* yi = L.ya + (i * Hb + k) * 2;
        double dx, dy, D2, au;
        if (j >= 0) {
            dx = pi[0] - L.pb[(j * Hb + k) * 2];
            dy = pi[1] - L.pb[(j * Hb + k) * 2 + 1];
            D2 = P.D2veh[i * SCPQP_MAX_VEH + j];
            const ldouble* yj = L.ya + (j * Hb + k) * 2;
            au = -2.0 * (dx * yi[0] + dy * yi[1]) + 2.0 * (dx * yj[0] + dy * yj[1]);
        } else {
            dx = pi[0] - L.ob[(o * Hb + k) * 2];
            dy = pi[1] - L.ob[(o * Hb + k) * 2 + 1];
            D2 = P.D2obs[i * SCPQP_MAX_OBST + o];
            au = -2.0 * (dx * yi[0] + dy * yi[1]);
        }
        const double c = D2 - (dx * dx + dy * dy);
        const double brow = -c + au;
        double a2 = 0.0;
        const ldouble* gi = L.g + i * Hb * 2;
        for (int l = 0; l <= k; ++l) {
            const double t = dx * gi[(k - l) * 2] + dy * gi[(k - l) * 2 + 1];
            a2 += t * t;
        }
        if (j >= 0) {
            const ldouble* gj = L.g + j * Hb * 2;
            for (int l = 0; l <= k; ++l) {
                const double t = dx * gj[(k - l) * 2] + dy * gj[(k - l) * 2 + 1];
                a2 += t * t;
            }
        }
        const double nrm = sqrt(4.0 * a2 * P.uLim * P.uLim + 1.0);
        L.rowE[2 * r] = 2.0 * dx * P.uLim / nrm;
        L.rowE[2 * r + 1] = 2.0 * dy * P.uLim / nrm;
        L.rowW[r] = -1.0 / nrm;
        L.rowH[r] = brow / nrm;
    }
    bar();
}

// ---------------------------------------------------------------------------
// QP: Mehrotra predictor-corrector IPM + active-set polish, scaled variables.
// x = L.z = [u~ (N), omega].  Returns IPM iterations; sets *qflags.
// ---------------------------------------------------------------------------
// out = G x (- h if minus_h)
template <class LT, class PX, class PO>
__device__ void g_apply(const LT& L, PX x, PO out, bool minus_h) {
    toeplitz_apply(L, x, L.ya);
    bar();
    const double xw = x[L.N];
    for (int r = threadIdx.x; r < L.mc; r += NT) {
        double val = gx_row(L, x, xw, r);
        if (minus_h) val -= hval(L, r);
        out[r] = val;
    }
    bar();
}

// residuals rd (n), rp (mc) at (z, s, lam); out = {max|rp|, max|rd|, gap, pobj}
template <class LT>
__device__ void residuals(const cParams& P, const LT& L, double (&out)[4]) {
    const int tid = threadIdx.x, N = L.N, Hb = L.Hb;
    const double u2 = P.uLim * P.uLim;
    toeplitz_apply(L, L.z, L.ya);
    bar();
    const double zw = L.z[N];
    double mrp = 0.0, gap = 0.0, wl = 0.0, quad = 0.0;
    for (int r = tid; r < L.mc; r += NT) {
        const double sr = L.s[r], lr = L.lam[r];
        const double v = gx_row(L, L.z, zw, r) + sr - hval(L, r);
        L.rp[r] = v;
        mrp = fmax(mrp, fabs(v));
        gap += sr * lr;
        if (r < L.m) wl += lr * L.rowW[r];
        // the next IPM iteration's weights d = lam / s and predictor vector
        // tv = d rp - (s lam) / s (round 5: formed here, in the thread that owns row r,
        // instead of two passes and two barriers of the factorisation phase)
        const double is = recip(sr), dr = lr * is;
        L.dd[r] = dr;
        L.tv[r] = dr * v - (sr * lr) * is;
    }
    for (int e = tid; e < L.V * Hb; e += NT) {
        const int v = e / Hb, k = e % Hb;
        const double qk = 2.0 * u2 * ((k == Hb - 1) ? P.Qf[v] : P.Q[v]);
        double s0, s1;
        incident_sum(L, v, k, [&](int r) { return L.lam[r]; }, s0, s1);
        const double y0 = L.ya[2 * e], y1 = L.ya[2 * e + 1];
        L.yb[2 * e] = qk * y0 + s0;
        L.yb[2 * e + 1] = qk * y1 + s1;
        quad += qk * (y0 * y0 + y1 * y1);
    }
    double red[4] = {mrp, gap, wl, quad};
    block_reduce4<4>(red, 1, L.red);
    double mrd = 0.0, quad2 = 0.0, lin = 0.0;
    toeplitz_t_apply(L, L.yb, [&](int e, double tt) {
        const int v = e / Hb;
        const double ze = L.z[e];
        const double pu = 2.0 * u2 * P.R[v] * ze;
        const double rde = tt + pu + L.qs[e] + L.lam[L.m + e] - L.lam[L.m + N + e];
        L.rd[e] = rde;
        mrd = fmax(mrd, fabs(rde));
        quad2 += pu * ze;
        lin += L.qs[e] * ze;
    });
    const double rdw = P.slackW + red[2] - L.lam[L.mc - 1];
    if (tid == 0) L.rd[N] = rdw;
    double red2[4] = {mrd, quad2, lin, 0.0};
    block_reduce4<3, 1>(red2, 1, L.red);
    out[0] = red[0];
    out[1] = fmax(red2[0], fabs(rdw));
    out[2] = red[1];
    out[3] = 0.5 * (red[3] + red2[1]) + red2[2] + P.slackW * zw;
}

// ---------------------------------------------------------------------------
// Phase functions.  Each is deliberately out of line and takes a 3-scalar
// context from which it rebuilds the LDS layout (a few integer ops), so every
// phase is register-allocated on its own and the IPM driver keeps only a few
// scalars live.  (One monolithic inlined body needed ~450 registers.)
// ---------------------------------------------------------------------------
struct Ctx {
    const cParams* P;
    gdouble* ws;
    int Hb, lead;
};
struct D4 {
    double a, b, c, d;
};

// Multiplier-iteration stopping rule of the polish (oracle POLISH_TOL): 1 once
// x stops moving (|dx| <= tol max(1, |x|)), 2 when the iterate shows the active
// set is wrong (warm rounds: a violated inactive row or a negative active
// multiplier beyond `early`), 0 to continue.  Never before the second solve.
constexpr double kPolishTol = 1e-9;
// The polish penalty (warm and cold rounds alike) is polish_delta; 1/delta of the
// current round lives in red[kIdlSlot] (set by the prep phases).  A separate warm
// penalty was measured and not kept.
__device__ __forceinline__ int polish_stop(const D4& d, int ref, double early) {
    if (ref < 1) return 0;
    if (d.a <= kPolishTol * fmax(1.0, d.b)) return 1;
    if (d.c > early || d.d > early) return 2;
    return 0;
}

// Out-of-line phases receive Ctx in VGPRs (the calling convention passes every
// argument per lane).  Its fields are workgroup-uniform: move them to SGPRs so
// that the parameter loads are scalar and every size, loop bound and offset
// derived from them stays scalar (SALU loop control, uniform branches).
__device__ __forceinline__ Ctx uniform_ctx(const Ctx& c) {
    Ctx u;
    u.P = (const cParams*)readfirstlane_u64((unsigned long long)c.P);
    u.ws = (gdouble*)readfirstlane_u64((unsigned long long)c.ws);
    u.Hb = __builtin_amdgcn_readfirstlane(c.Hb);
    u.lead = __builtin_amdgcn_readfirstlane(c.lead);
    return u;
}

template <bool HG, bool VG, int RM, int OCC, int SH>
__device__ __forceinline__ Lay<HG, VG, RM, OCC> lay_of(const Ctx& c) {
    const Off f = plan_offsets(shapeV<SH>(c.P->nV), shapeO<SH>(c.P->nO), shapeHM<SH>(c.P->hpMax), HG, VG, lean_plan(HG, VG, OCC));
    Lay<HG, VG, RM, OCC> L = make_lay<HG, VG, RM, OCC, SH>((ldouble*)smem_, c.ws, f, c.P->nV, c.P->nO, c.Hb);
    L.lead = c.lead;
    return L;
}
#define PHASE template <bool HG, bool VG, int RM, int OCC, int SH> __device__ __noinline__
#define LAYDEF                  \
    const Ctx cu_ = uniform_ctx(c); \
    const cParams& P = *cu_.P;  \
    const Lay<HG, VG, RM, OCC> L = lay_of<HG, VG, RM, OCC, SH>(cu_); \
    (void)P
#define PH(f) f<HG, VG, RM, OCC, SH>

// x = K^{-1} rhs into z (dst = 0) or dz (dst = 1)
PHASE void ph_solve(Ctx c, int dst) {
    LAYDEF;
    chol_solve<SH>(L, L.rhs, dst ? L.dz : L.z);
}
PHASE void ph_linearise(Ctx c) {
    LAYDEF;
    linearise_rows(P, L);
}
PHASE EvalRes ph_evaluate(Ctx c, double* cveh, double* cobs) {
    LAYDEF;
    return evaluate_u(P, L, L.ub, cveh, cobs);
}
PHASE D4 ph_residuals(Ctx c) {
    LAYDEF;
    double r[4];
    residuals(P, L, r);
    return D4{r[0], r[1], r[2], r[3]};
}
// rhs = -q + G'(tv) with tv = h (init) or tv = mask (h/delta - y) (polish), + rho x_k.
// Buffer 1: in ph_polish_dual_next it follows polish_dual_body's reduction (buffer 0)
// with no barrier between them; its other callers reach it after a barrier.
template <class LT>
__device__ __forceinline__ void rhs_from_tv_body(const cParams& P, const LT& L, double rho) {
    const double ow = gt_apply_fin<1>(L, L.tv, [&](int e, double g) { L.rhs[e] = g - L.qs[e] + rho * L.dz[e]; });
    if (threadIdx.x == 0) L.rhs[L.N] = ow - P.slackW + rho * L.dz[L.N];
    bar();
}
PHASE void ph_rhs_from_tv(Ctx c, double rho) {
    LAYDEF;
    rhs_from_tv_body(P, L, rho);
}
// initial-point setup of dd/tv/dz
PHASE void ph_init_a(Ctx c) {
    LAYDEF;
    const int tid = threadIdx.x;
    for (int r = tid; r < L.mc; r += NT) {
        L.dd[r] = 1.0;
        L.tv[r] = hval(L, r);
    }
    for (int e = tid; e < L.n; e += NT) L.dz[e] = 0.0;
    bar();
}
// Initial point (round 3).  The CVXOPT point below starts the slack omega from the
// normal system, where its weight (1e5, SCP_controller.py:138) drives it to -1e4 and
// the multipliers to 1e5 spread over every row; the iterates then crawl for 5-8
// iterations with steps of 0.1-0.4 (tools/ipm_corrector_study.py).  Instead:
//  * the controls solve the omega-free normal system (row N of P + G'G decoupled:
//    ph_init_assemble_factor between the assembly and the factorisation);
//  * omega = the smallest value that satisfies every collision row, plus one;
//  * s = h - G x, shifted positive (1.5 x its most negative entry) and floored at a
//    tenth of its largest entry;
//  * lam = 0.3 slackW / mc on every row, slackW on the omega bound (whose multiplier
//    carries the slack weight at any point with omega = 0).
// CPU study, cold IPM iterations per QP (tools/ipm_corrector_study.py): c2 15.7 -> 12.5,
// 4 veh Hp 10 14.3 -> 10.1, Hp 30 16.0 -> 13.0, parallel5 23.1 -> 18.0, frog 16.7 -> 14.7;
// every QP's polish certifies the same minimiser.  (CVXOPT's own point, and starting the
// controls at 0 without the initial solve, were measured and not kept: DESIGN §3.)
PHASE void ph_init_b(Ctx c) {
    LAYDEF;
    const int tid = threadIdx.x, N = L.N, mc = L.mc;
    toeplitz_apply(L, L.z, L.ya);
    bar();
    double vmax = 0.0;
    for (int r = tid; r < L.m; r += NT) {
        const double gu = gx_row(L, L.z, 0.0, r);
        L.s[r] = gu;
        vmax = fmax(vmax, (gu - L.rowH[r]) / -L.rowW[r]);
    }
    double red[4] = {vmax, 0.0, 0.0, 0.0};
    block_reduce4<1>(red, 1, L.red);
    const double om = red[0] + 1.0;
    double smin = 1e300, smax = -1e300;
    for (int r = tid; r < mc; r += NT) {
        const double gx = r < L.m ? L.s[r] + L.rowW[r] * om : gx_row(L, L.z, om, r);
        const double sv = hval(L, r) - gx;
        L.s[r] = sv;
        smin = fmin(smin, sv);
        smax = fmax(smax, sv);
    }
    double red2[4] = {-smin, smax, 0.0, 0.0};
    block_reduce4<2, 1>(red2, 3, L.red);
    const double ts = fmax(1.5 * red2[0], 0.0);
    const double fl = 0.1 * fmax(1.0, red2[1] + ts);
    const double lam0 = 0.3 * P.slackW / mc;
    for (int r = tid; r < mc; r += NT) {
        L.s[r] = fmax(L.s[r] + ts, fl);
        L.lam[r] = r == mc - 1 ? P.slackW : lam0;
    }
    if (tid == 0) L.z[N] = om;
    bar();
}
// Interior-point step bodies.  The phase functions below chain several of
// them in one out-of-line call: every call costs its register save/restore
// and layout rebuild (~2k cycles for a trivial phase), and the bodies of one
// chain touch the same rows from the same threads.
//
// Newton direction, complementarity target rc = s lam (+ ds_aff dl_aff - smu if corr):
//   rhs = -rd - G'(d rp - rc/s);  dz = K^{-1} rhs;  ds = -rp - G dz;  dl = -(rc + lam ds)/s
template <bool TV = true, class LT>
__device__ __forceinline__ void newton_rhs_body(const LT& L, int corr, double smu) {
    if constexpr (TV) {   // else tv is already formed (the predictor: residuals())
        for (int r = threadIdx.x; r < L.mc; r += NT) {
            const double rc = L.s[r] * L.lam[r] + (corr ? L.sa[r] * L.la[r] - smu : 0.0);
            L.tv[r] = L.dd[r] * L.rp[r] - rc * recip(L.s[r]);
        }
        bar();
    }
    // buffer 0: reached after assemble's closing barrier or the tv pass's barrier
    const double ow = gt_apply_fin<0>(L, L.tv, [&](int e, double g) { L.rhs[e] = -L.rd[e] - g; });
    if (threadIdx.x == 0) L.rhs[L.N] = -L.rd[L.N] - ow;
    bar();
}
// ds = -rp - G dz row by row in the thread that forms (G dz)_r, and this thread's
// partial step lengths {primal: min over ds < 0 of -s/ds, dual: min over dl < 0 of
// -lam/dl} from the values it just formed (round 5: one barrier and one pass over the
// rows fewer than G dz, the direction and the ratio tests apart; the same operations).
template <class LT>
__device__ __forceinline__ double2v newton_back_body(const LT& L, int corr, double smu) {
    toeplitz_apply(L, L.dz, L.ya);
    bar();
    const double xw = L.dz[L.N];
    double ap = 1.0, ad = 1.0;
    for (int r = threadIdx.x; r < L.mc; r += NT) {
        const double rc = L.s[r] * L.lam[r] + (corr ? L.sa[r] * L.la[r] - smu : 0.0);
        const double dsr = -L.rp[r] - gx_row(L, L.dz, xw, r);
        const double dlr = -(rc + L.lam[r] * dsr) * recip(L.s[r]);
        L.ds[r] = dsr;
        L.dl[r] = dlr;
        if (dsr < 0.0) ap = fmin(ap, -L.s[r] * recip(dsr));
        if (dlr < 0.0) ad = fmin(ad, -L.lam[r] * recip(dlr));
    }
    bar();
    return double2v{ap, ad};
}
// predictor step length and Mehrotra centring: returns sigma * mu; stores the affine direction
template <class LT>
__device__ __forceinline__ double affine_body(const LT& L, double mu, double2v part) {
    double redm[4] = {-fmin(part.x, part.y), 0.0, 0.0, 0.0};
    block_reduce4<1>(redm, 1, L.red);   // = max_step(L)
    const double aaff = -redm[0];
    double mua = 0.0;
    for (int r = threadIdx.x; r < L.mc; r += NT) {
        mua += (L.s[r] + aaff * L.ds[r]) * (L.lam[r] + aaff * L.dl[r]);
        L.sa[r] = L.ds[r];
        L.la[r] = L.dl[r];
    }
    double red[4] = {mua, 0.0, 0.0, 0.0};
    block_reduce4<1, 1>(red, 0, L.red);   // follows max_step's (buffer 0)
    const double sr = red[0] / L.mc / mu;
    return sr * sr * sr * mu;
}
// Separate primal and dual step lengths (round 3): (z, s) move by the primal ratio test
// and lam by the dual one, each damped by step_factor.  The QP's dual residual is then no
// longer scaled by (1 - a) exactly (P couples it to the primal step), which the next
// iteration's residuals absorb.  CPU study, cold IPM iterations per QP: c2 11.4 -> 10.9,
// Hp 30 11.0 -> 10.1, c3 14.0 -> 13.1 (max 23 -> 19), frog 15.9 -> 11.0; Hp 10 and
// parallel5 unchanged; every polish certifies the same minimiser.
template <class LT>
__device__ __forceinline__ void update_body(const LT& L, double eta, double2v part) {
    // separate step lengths: (z, s) by the primal ratio test, lam by the dual one
    double ap = part.x, ad = part.y;
    double red[4] = {-ap, -ad, 0.0, 0.0};
    block_reduce4<2>(red, 3, L.red);
    ap = fmin(1.0, eta * -red[0]);
    ad = fmin(1.0, eta * -red[1]);
    for (int e = threadIdx.x; e < L.n; e += NT) L.z[e] += ap * L.dz[e];
    for (int r = threadIdx.x; r < L.mc; r += NT) {
        L.s[r] += ap * L.ds[r];
        L.lam[r] += ad * L.dl[r];
    }
    bar();
}
// Fraction of the step to the boundary (round 3): max(0.99, 1 - mu) instead of a fixed
// 0.99, i.e. nearly full steps once the scaled complementarity is small.  CPU study
// (tools/ipm_corrector_study.py, from the round-3 start): cold IPM iterations per QP
// c2 12.5 -> 11.5, 4 veh Hp 10 10.1 -> 7.8, parallel5 18.0 -> 16.6, frog 14.7 -> 12.0.
__device__ __forceinline__ double step_factor(double mu) { return fmax(0.99, 1.0 - mu); }
// d = lam / s, K = P + G' diag(d) G, the predictor right-hand side (rc = s lam; it does
// not need the factor, so it is formed before the factorisation) and L D L' of K in one
// call (one call fewer per IPM iteration than assembly and factorisation apart: c2 +0.8 %,
// profiles/r03_ab_fuse_fact.txt).  1 = factored.
// d and tv come from the residuals of this iterate (residuals()), which every IPM
// iteration computes last and every IPM pass first.
PHASE int ph_scale_assemble_rhs_factor(Ctx c) {
    LAYDEF;
    PROF_T0_FINE();
    assemble(P, L, L.dd, 0.0);
    PROF_ACC_FINE0(29);
    newton_rhs_body<false>(L, 0, 0.0);
    PROF_ACC_FINE0(28);
    return cholesky(L) ? 1 : 0;
}
// polish: K = P + rho I + G_A' G_A / delta, factored in the same call
PHASE int ph_assemble_factor(Ctx c, double rho) {
    LAYDEF;
    assemble(P, L, L.dd, rho);
    return cholesky(L) ? 1 : 0;
}
// the cold IPM's starting system P + G'G with its omega row decoupled (row N = e_N),
// assembled and factored in one call
PHASE void ph_init_assemble_factor(Ctx c) {
    LAYDEF;
    assemble(P, L, L.dd, 0.0);
    const int N = L.N, o = roff(N);
    for (int e = threadIdx.x; e <= N; e += NT) L.H[o + e] = e == N ? 1.0 : 0.0;
    bar();
    cholesky(L);   // P + G'G is positive definite (box and omega rows)
}
// predictor back-substitution, affine step and centring, corrector right-hand side
PHASE double ph_back_affine_rhs(Ctx c, double mu) {
    LAYDEF;
    const double2v part = newton_back_body(L, 0, 0.0);
    const double smu = affine_body(L, mu, part);
    newton_rhs_body(L, 1, smu);
    return smu;
}
// corrector back-substitution, the damped step, and the residuals of the new
// point (the next iteration's convergence test)
PHASE D4 ph_back_update_residuals(Ctx c, double smu, double eta) {
    LAYDEF;
    const double2v part = newton_back_body(L, 1, smu);
    update_body(L, eta, part);
    double r[4];
    residuals(P, L, r);
    return D4{r[0], r[1], r[2], r[3]};
}
// polish: weights 1/delta on the active set {lam > s}, y = lam there, x_0 = z
PHASE void ph_polish_prep(Ctx c) {
    LAYDEF;
    const double idl = 1.0 / P.polDelta;
    if (threadIdx.x == 0) L.red[kIdlSlot] = idl;
    for (int r = threadIdx.x; r < L.mc; r += NT) {
        const bool act = L.lam[r] > L.s[r];
        L.dd[r] = act ? idl : 0.0;
        L.la[r] = act ? L.lam[r] : 0.0;   // y
        L.sa[r] = act ? 1.0 : 0.0;        // active mask
    }
    for (int e = threadIdx.x; e < L.n; e += NT) L.dz[e] = L.rd[e] = L.z[e];
    bar();
}
// warm start from the previous QP of this problem: its active set (sa) and
// multipliers (la) on the re-linearised rows, x_0 = its solution (z)
PHASE void ph_polish_warm(Ctx c) {
    LAYDEF;
    const double idl = 1.0 / P.polDelta;
    if (threadIdx.x == 0) L.red[kIdlSlot] = idl;
    for (int r = threadIdx.x; r < L.mc; r += NT) L.dd[r] = L.sa[r] != 0.0 ? idl : 0.0;
    for (int e = threadIdx.x; e < L.n; e += NT) L.dz[e] = L.rd[e] = L.z[e];
    bar();
}
// termination-test scales: max(1, |h|), max(1, slack weight, |q|)
PHASE D4 ph_scales(Ctx c) {
    LAYDEF;
    const int tid = threadIdx.x;
    double hmax = 1.0;
    for (int r = tid; r < L.m; r += NT) hmax = fmax(hmax, fabs(L.rowH[r]));
    double qmax = fmax(1.0, P.slackW);
    for (int e = tid; e < L.N; e += NT) qmax = fmax(qmax, fabs(L.qs[e]));
    double red[4] = {hmax, qmax, 0.0, 0.0};
    block_reduce4<2>(red, 3, L.red);
    return D4{red[0], red[1], 0.0, 0.0};
}
// polish right-hand side: tv = mask (h / delta - y), rhs = -q + G' tv + rho x_k
template <class LT>
__device__ __forceinline__ void polish_rhs_body(const cParams& P, const LT& L) {
    const double idl = L.red[kIdlSlot];
    for (int r = threadIdx.x; r < L.mc; r += NT) L.tv[r] = L.sa[r] * (hval(L, r) * idl - L.la[r]);
    bar();
    rhs_from_tv_body(P, L, P.polRho);
}
PHASE void ph_polish_rhs(Ctx c) {
    LAYDEF;
    polish_rhs_body(P, L);
}
// rp = G x_k - h;  y += rp / delta on the active set.  Returns
// {max |x_k - x_{k-1}|, max |x_k|, max rp over the inactive rows, -min y over
// the active rows} (x_{k-1} kept in rd, dead during the polish).
template <class LT>
__device__ __forceinline__ D4 polish_dual_body(const cParams& P, const LT& L) {
    const double idl = L.red[kIdlSlot];
    // rp = G x_k - h row by row in the thread that uses it (round 5: one barrier fewer
    // per multiplier iteration than G x_k - h and the update apart)
    toeplitz_apply(L, L.dz, L.ya);
    bar();
    const double xw = L.dz[L.N];
    double viol = -1e300, yneg = -1e300;
    for (int r = threadIdx.x; r < L.mc; r += NT) {
        const double hr = hval(L, r);
        const double rpr = gx_row(L, L.dz, xw, r) - hr;
        L.rp[r] = rpr;
        const double sar = L.sa[r];
        double y = L.la[r];
        if (sar != 0.0) {
            y = y + rpr * idl;
            L.la[r] = y;
            yneg = fmax(yneg, -y);
        } else {
            viol = fmax(viol, rpr);
        }
        // the next refinement's tv = mask (h / delta - y) (polish_rhs_body), formed here
        // in the row's own thread: its pass and barrier leave the multiplier iteration
        L.tv[r] = sar * (hr * idl - y);
    }
    double dmax = 0.0, xmax = 0.0;
    for (int e = threadIdx.x; e < L.n; e += NT) {
        const double x = L.dz[e];
        dmax = fmax(dmax, fabs(x - L.rd[e]));
        xmax = fmax(xmax, fabs(x));
        L.rd[e] = x;
    }
    double red[4] = {dmax, xmax, viol, yneg};
    block_reduce4<4>(red, 15, L.red);
    return D4{red[0], red[1], red[2], red[3]};
}
// the multiplier update, and, unless the caller's stopping rule (polish_stop)
// ends the refinement here, the next right-hand side in the same call
PHASE D4 ph_polish_dual_next(Ctx c, int ref, int cap, double early) {
    LAYDEF;
    const D4 d = polish_dual_body(P, L);
    if (polish_stop(d, ref, early) == 0 && ref + 1 < cap) rhs_from_tv_body(P, L, P.polRho);
    return d;
}
// certify the polished point (primal feasible, y >= 0, finite); accept -> z.
// Otherwise one primal-dual active-set correction (oracle _pdas_update): add the
// violated inactive rows, drop the active rows with negative multipliers, and
// rebuild the polish weights.  Returns 1 accepted, 1 + (rows changed) >= 2
// corrected (retry), 0 stuck.
PHASE int ph_polish_accept(Ctx c, double hmax, int converged) {
    LAYDEF;
    const int tid = threadIdx.x;
    double viol = -1e300, ymin = 1e300, ymax = 0.0, nonfin = 0.0;
    for (int r = tid; r < L.mc; r += NT) {
        viol = fmax(viol, L.rp[r]);
        if (L.sa[r] != 0.0) {
            ymin = fmin(ymin, L.la[r]);
            ymax = fmax(ymax, fabs(L.la[r]));
        }
    }
    for (int e = tid; e < L.n; e += NT)
        if (!isfinite(L.dz[e])) nonfin = 1.0;
    double red[4] = {viol, -ymin, ymax, nonfin};
    block_reduce4<4, 1>(red, 15, L.red);   // may follow polish_dual_body's (buffer 0)
    const double vtol = 1e-9 * hmax, ytol = -1e-9 * fmax(1.0, red[2]);
    // a point is certified only if the multiplier iteration has also converged
    // (stationarity), else only the active set is corrected
    const bool ok = converged && red[0] <= vtol && -red[1] >= ytol && red[3] == 0.0;
    if (ok) {
        for (int e = tid; e < L.n; e += NT) L.z[e] = L.dz[e];
        bar();
        return 1;
    }
    if (red[3] != 0.0) return 0;
    const double idl = L.red[kIdlSlot];
    double changed = 0.0;
    for (int r = tid; r < L.mc; r += NT) {
        const bool act = L.sa[r] != 0.0;
        const bool add = !act && L.rp[r] > vtol;
        const bool drop = act && L.la[r] < ytol;
        if (add || drop) {
            changed += 1.0;
            L.sa[r] = add ? 1.0 : 0.0;
            L.la[r] = 0.0;
            L.dd[r] = add ? idl : 0.0;
        }
    }
    double red2[4] = {changed, 0.0, 0.0, 0.0};
    block_reduce4<1>(red2, 0, L.red);
    return red2[0] != 0.0 ? 1 + (int)red2[0] : 0;
}
// u-bar <- uLim * z  (unscaled controls of the QP solution)
PHASE void ph_take_u(Ctx c) {
    LAYDEF;
    for (int i = threadIdx.x; i < L.N; i += NT) L.ub[i] = P.uLim * L.z[i];
    bar();
}

// Per-iteration trace (scpqp_batch_out.trace), written only when requested.
// Before take_u: the linearisation point u-bar and the factored rows it gave.
PHASE void ph_trace_rows(Ctx c, double* dst) {
    LAYDEF;
    for (int i = threadIdx.x; i < L.N; i += NT) dst[kTraceHdr + i] = L.ub[i];
    const int N2 = kTraceHdr + 2 * P.nV * P.hpMax;
    for (int r = threadIdx.x; r < L.m; r += NT) {
        dst[N2 + 4 * r] = L.rowE[2 * r];
        dst[N2 + 4 * r + 1] = L.rowE[2 * r + 1];
        dst[N2 + 4 * r + 2] = L.rowW[r];
        dst[N2 + 4 * r + 3] = L.rowH[r];
    }
}
// After the evaluation: the QP's solution, its slack and the stopping-rule terms.
PHASE void ph_trace_sol(Ctx c, double* dst, D4 ev, double delta, int ipm, int qfl, double merit0,
                        int rounds, int refines) {
    LAYDEF;
    for (int i = threadIdx.x; i < L.N; i += NT) dst[kTraceHdr + P.nV * P.hpMax + i] = L.ub[i];
    if (threadIdx.x == 0) {
        dst[8] = merit0;   // obj_0 + 1e5 max_violation_0 before this iteration (delta_hat, :159)
        dst[9] = rounds + 4096.0 * refines;   // this QP's polish rounds and refinement solves
        dst[0] = delta;
        dst[1] = ev.a;
        dst[2] = ev.b;
        dst[3] = ev.c;
        dst[4] = L.z[L.N];
        dst[5] = ipm;
        dst[6] = qfl;
        dst[7] = ev.d;
    }
}

// Active-set corrections of the polish (oracle POLISH_ROUNDS), the rounds a
// warm start may take before the IPM runs, and the multiplier iteration's
// convergence test (oracle POLISH_TOL).
constexpr int kPolishRounds = 6;
constexpr int kWarmRounds = 8;        // 4 measured within noise or slower
constexpr int kWarmRefine = 12;       // solve cap per warm round (cold rounds: P.nRefine)
// Warm rounds stop refining as soon as the iterate shows the active set is
// wrong (an inactive row violated, or an active multiplier negative, by more
// than this in scaled units): the correction comes earlier and the refinement
// spent on a wrong active set is skipped.
constexpr double kWarmEarly = 1e-6;
// A warm start whose active-set corrections stop shrinking is abandoned for the
// cold IPM.  On c3 half the warm starts fail, each after all kWarmRounds
// refactorisations, and a round costs as much as an IPM iteration (c3 4.45k ->
// 4.79k solves/s).  At the round-1 polish stopping tolerance the late warm rounds
// of c2-size problems still certified often enough that the rule cost c2 1-2 %
// (tools/warm_policy_study.py); with the 1e-9 tolerance it gains c2 2-3 %
// (profiles/r02_ab_warm_stall.txt), so it applies to every plan.
constexpr bool kWarmStall = true;

// ---------------------------------------------------------------------------
// QP driver: Mehrotra predictor-corrector IPM + active-set polish (scaled
// variables, x = z = [u~ (N), omega]).  Returns IPM iterations; sets *qflags.
// ---------------------------------------------------------------------------
struct QpStats {
    int ipm, rounds, refine, warm_ok;
};

// Polish rounds: proximal method of multipliers on the active set in sa/la/dd,
// refined until x stops moving (|dx| <= kPolishTol max(1, |x|), at most
// P.nRefine solves per round), certified, else the active set is corrected
// (primal-dual active set) and the round repeats.  Returns true if certified.
// stall: give up once a correction changes no fewer rows than the one before
// (warm rounds, see kWarmStall).
template <bool HG, bool VG, int RM, int OCC, int SH>
__device__ __forceinline__ bool polish_rounds(Ctx c, double hmax, double rho, int max_rounds,
                                              int cap, double early, QpStats& st, bool stall = false) {
    bool ok = false, refactor = true, extended = false;
    int prev_chg = 1 << 30;
    PROF_T0();
    for (int round = 0; round < max_rounds && !ok; ++round) {
        ++st.rounds;
        if (refactor) {
            const bool fact = PH(ph_assemble_factor)(c, rho) != 0;
            PROF_ACC(7);
            if (!fact) break;
        }
        int conv = 0;
        PH(ph_polish_rhs)(c);
        for (int ref = 0; ref < cap; ++ref) {
            PH(ph_solve)(c, 1);
            const D4 d = PH(ph_polish_dual_next)(c, ref, cap, early);
            ++st.refine;
            const int stop = polish_stop(d, ref, early);
            conv = stop == 1;
            if (stop) break;
        }
        const int acc = PH(ph_polish_accept)(c, hmax, conv);
        PROF_ACC(8);
        ok = acc == 1;
        // acc >= 2: active set corrected -> refactor;  acc 0 with the multiplier
        // iteration still moving: same active set, keep iterating on the same
        // factor;  acc 0 after convergence: stuck, give up
        if (acc == 0 && (conv || extended)) break;
        if (acc >= 2) {
            if (stall && round >= 1 && acc - 1 >= prev_chg) break;
            prev_chg = acc - 1;
        }
        extended |= acc == 0;   // one extra batch of iterations per QP
        refactor = acc >= 2;
    }
    return ok;
}

// One convexified QP.  warm: try the previous QP's active set first (a few
// polish rounds, no interior point iterations); on failure, or cold, run the
// Mehrotra IPM from the CVXOPT initial point and polish its active set.
// The driver keeps its counters and the parameters its loops test in
// registers: the callers' QpStats/flags live on the private stack, and a
// parameter re-read after every out-of-line phase is a global-memory load on
// the iteration's critical path.
struct QpKnobs {
    int maxIpm, nRefine, mc;
    double ipmTol, polRho;
};
template <bool HG, bool VG, int RM, int OCC, int SH>
__device__ __forceinline__ bool qp_solve_body(Ctx c, const QpKnobs& K, int& qflags, bool warm,
                                              QpStats& st) {
    const int mc = K.mc;
    const D4 sc = PH(ph_scales)(c);
    const double hmax = sc.a, qmax = sc.b;
    if (warm) {
        PH(ph_polish_warm)(c);
        if (polish_rounds<HG, VG, RM, OCC, SH>(c, hmax, K.polRho, kWarmRounds, kWarmRefine, kWarmEarly,
                                               st, kWarmStall)) {
            ++st.warm_ok;
            return true;
        }
    }
    // ---- initial point: (P + G'G) x = -q + G'h (omega decoupled, see ph_init_b);
    // s = h - Gx and lam from ph_init_b
    PROF_T0();
    PH(ph_init_a)(c);
    PH(ph_init_assemble_factor)(c);
    PH(ph_rhs_from_tv)(c, 0.0);
    PH(ph_solve)(c, 0);
    PH(ph_init_b)(c);
    PROF_ACC(16);
    // ---- Mehrotra iterations
    int it = 0;
    bool conv = false, ok = false, maxit = false;
    double tol = K.ipmTol;
    D4 res = PH(ph_residuals)(c);
    PROF_ACC(1);
    for (int pass = 0;; ++pass) {
        for (; it < K.maxIpm; ++it) {
            PROF_ACC(0);
            if (res.a <= tol * hmax && res.b <= tol * qmax && res.c <= tol * fmax(1.0, fabs(res.d))) {
                conv = true;
                break;
            }
            const double mu = res.c / mc;
            if (!PH(ph_scale_assemble_rhs_factor)(c)) break;
            PROF_ACC(3);
            PH(ph_solve)(c, 1);
            PROF_ACC(9);
            const double smu = PH(ph_back_affine_rhs)(c, mu);
            PROF_ACC(5);
            PH(ph_solve)(c, 1);
            PROF_ACC(9);
            res = PH(ph_back_update_residuals)(c, smu, step_factor(mu));
            PROF_ACC(6);
        }
        // the iteration cap counts against the QP only in the first pass: a resumed pass
        // (below) runs 100x tighter than the QP's tolerance, which it has already met
        if (pass == 0 && !conv && it >= K.maxIpm) maxit = true;
        // ---- active-set polish on {lam > s}
        PH(ph_polish_prep)(c);
        ok = polish_rounds<HG, VG, RM, OCC, SH>(c, hmax, K.polRho, kPolishRounds, K.nRefine, INFINITY, st);
        // The dual residual is measured against max(1, slackW, |q|) = 1e5, so a point that
        // passes the tolerance can still leave weakly active rows undecided and the polish
        // uncertified (the c3 golden's third QP from the round-3 starting point: 6e-6 rad
        // off).  The polish leaves (z, s, lam) untouched: resume the IPM 100x tighter (in
        // practice until the normal matrix breaks down, one or two iterations) and polish
        // once more.
        if (ok || !conv || pass == 1) break;
        tol *= 0.01;
        conv = false;
        res = PH(ph_residuals)(c);
    }
    st.ipm += it;
    if (maxit) qflags |= SCPQP_FL_IPM_MAXIT;
    if (!ok) qflags |= SCPQP_FL_POLISH_REJECTED;
    return ok;
}
template <bool HG, bool VG, int RM, int OCC, int SH>
__device__ __noinline__ bool qp_solve(Ctx c0, int* qflags, bool warm, QpStats& st) {
    const Ctx c = uniform_ctx(c0);
    const cParams& P = *c.P;
    QpKnobs K;
    K.maxIpm = __builtin_amdgcn_readfirstlane(P.maxIpm);
    K.nRefine = __builtin_amdgcn_readfirstlane(P.nRefine);
    K.mc = __builtin_amdgcn_readfirstlane(
        (P.nV * (P.nV - 1) / 2 + P.nV * P.nO) * c.Hb + 2 * P.nV * c.Hb + 1);
    K.ipmTol = P.ipmTol;
    K.polRho = P.polRho;
    QpStats ls{0, 0, 0, 0};
    int lf = 0;
    const bool ok = qp_solve_body<HG, VG, RM, OCC, SH>(c, K, lf, warm, ls);
    st.ipm += ls.ipm;
    st.rounds += ls.rounds;
    st.refine += ls.refine;
    st.warm_ok += ls.warm_ok;
    *qflags |= lf;
    return ok;
}

// ---------------------------------------------------------------------------
// Kernel
// ---------------------------------------------------------------------------
// Lead election: one counter per CU (XCC, SE, SH, CU from the hardware
// registers); the k-th workgroup of a launch on a CU takes the wave that sits on
// SIMD k mod 4.  The persistent workgroups stay resident for the whole launch,
// and the counters only ever grow, so consecutive launches keep handing out
// consecutive SIMDs.  A placement heuristic only: any lead is correct.
__device__ unsigned g_cu_ctr[4096];
__device__ __forceinline__ int lead_wave_elect(lint* sh) {
    const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);    // HW_REG_HW_ID
    const unsigned xcc = __builtin_amdgcn_s_getreg((3 << 11) | 20);   // HW_REG_XCC_ID [3:0]
    const int simd = (hw >> 4) & 3;
    if (threadIdx.x == 0) {
        const unsigned key = ((xcc & 15) << 8) | (((hw >> 13) & 7) << 5) | (((hw >> 12) & 1) << 4) |
                             ((hw >> 8) & 15);
        sh[0] = atomicAdd(&g_cu_ctr[key], 1u) & 3;
        sh[1] = 0;
    }
    bar();
    if ((threadIdx.x & 63) == 0 && simd == sh[0]) sh[1] = threadIdx.x >> 6;
    bar();
    const int lead = __builtin_amdgcn_readfirstlane(sh[1]);
    bar();
    return lead;
}

template <bool HG, bool VG, int RM, int OCC, int SH>
__global__ __launch_bounds__(NT, OCC) void scp_kernel(KArgs a) {
    ldouble* smem = (ldouble*)smem_;
    const cParams& P = *(const cParams*)a.P;
    const int tid = threadIdx.x;
    gdouble* ws = a.ws ? (gdouble*)a.ws + (size_t)blockIdx.x * a.wsStride : nullptr;
    const Off f = plan_offsets(shapeV<SH>(P.nV), shapeO<SH>(P.nO), shapeHM<SH>(P.hpMax), HG, VG, lean_plan(HG, VG, OCC));
    lint* slot = (lint*)(smem + f.red + kWorkSlot);
    lint* orslot = (lint*)(smem + f.red + kOrSlot);
    ldouble* lub = smem + f.ub;   // u-bar
    ldouble* lpb = smem + f.pb;   // positions of the last evaluated u
    ldouble* lref = smem + f.ref;
    ldouble* lg = smem + f.g;
    ldouble* lp0 = smem + f.p0;
    ldouble* lqs = smem + f.qs;
    const int lead = lead_wave_elect((lint*)(smem + f.red + kLeadSlot));
    for (;;) {
        if (tid == 0) {
            const int w = atomicAdd(a.counter, 1);
            slot[0] = (a.perm && w < a.B) ? a.perm[w] : w;
        }
        bar();
        // problem index and horizon are workgroup-uniform: make them scalar so
        // every branch below that guards a barrier is a uniform (SALU) branch
        const int b = __builtin_amdgcn_readfirstlane(slot[0]);
        bar();
        if (b >= a.B) break;
        const int Hb = __builtin_amdgcn_readfirstlane(a.hp ? a.hp[b] : P.hpMax);
        if (Hb < 1 || Hb > P.hpMax) {   // horizon outside the slot: report, never index with it
            if (tid == 0) {
                if (a.status) a.status[b] = SCPQP_ST_INVALID;
                if (a.nscp) a.nscp[b] = 0;
                if (a.nipm) a.nipm[b] = 0;
                if (a.npol) a.npol[b] = 0;
                if (a.nref) a.nref[b] = 0;
                if (a.nwarm) a.nwarm[b] = 0;
            }
            bar();
            continue;
        }
        const Ctx c{(const cParams*)a.P, ws, Hb, lead};
        const int V = P.nV, N = V * Hb, O = P.nO;
#ifdef SCPQP_PROF
        if (tid == 0 && b < 8192) g_ptime[2 * b] = __builtin_amdgcn_s_memrealtime();
#endif
        PROF_T0();
        // the sampler's flags, ORed over the workgroup in an LDS slot (__syncthreads_or
        // would add 256 B of static LDS to every plan)
        if (tid == 0) *orslot = 0;
        const int sflag = setup_problem_ni<HG, VG, RM, OCC, SH>((const cKArgs*)__builtin_amdgcn_kernarg_segment_ptr(), ws, b, Hb);
        PROF_ACC(10);
        if (sflag) *orslot = 1;
        bar();
        const int sflag_any = *orslot;
        const size_t slotU = (size_t)b * V * P.hpMax;   // [B][V*Hmax] slots
        if (a.mode == MODE_SAMPLE) {
            for (int i = tid; i < Hb * 2 * V; i += NT) {
                const int k = i / (2 * V), cc = (i / V) & 1, v = i % V;
                a.refOut[(size_t)b * P.hpMax * 2 * V + i] = lref[(v * Hb + k) * 2 + cc];
            }
            continue;
        }
        if (a.mode == MODE_LINEARIZE) {
            for (int i = tid; i < V * Hb * 2; i += NT) {
                if (a.gOut) a.gOut[slotU * 2 + i] = lg[i];
                if (a.p0Out) a.p0Out[slotU * 2 + i] = lp0[i];
            }
            for (int i = tid; i < N; i += NT)
                if (a.psiOut) a.psiOut[slotU + i] = lqs[i] / P.uLim;
            if (a.refOut)
                for (int i = tid; i < Hb * 2 * V; i += NT) {
                    const int k = i / (2 * V), cc = (i / V) & 1, v = i % V;
                    a.refOut[(size_t)b * P.hpMax * 2 * V + i] = lref[(v * Hb + k) * 2 + cc];
                }
            bar();
            continue;
        }
        if (a.mode == MODE_EVALUATE) {
            for (int i = tid; i < N; i += NT) lub[i] = a.uEval[slotU + i];
            double* cv = a.cveh ? a.cveh + (size_t)b * V * V * P.hpMax : nullptr;
            double* co = a.cobs ? a.cobs + (size_t)b * V * O * P.hpMax : nullptr;
            if (cv)
                for (int i = tid; i < V * V * Hb; i += NT) cv[i] = -INFINITY;
            if (co)
                for (int i = tid; i < V * O * Hb; i += NT) co[i] = -INFINITY;
            bar();
            const EvalRes ev = PH(ph_evaluate)(c, cv, co);
            if (tid == 0) {
                if (a.obj) a.obj[b] = ev.obj;
                if (a.maxv) a.maxv[b] = ev.maxv;
                if (a.sumv) a.sumv[b] = ev.sumv;
                if (a.feas) a.feas[b] = ev.feasible;
            }
            if (a.trajOut)
                for (int i = tid; i < Hb * 2 * V; i += NT) {
                    const int k = i / (2 * V), cc = (i / V) & 1, v = i % V;
                    a.trajOut[(size_t)b * P.hpMax * 2 * V + i] = lpb[(v * Hb + k) * 2 + cc];
                }
            bar();
            continue;
        }
        // ------------------------------- SCP solve (SCP_controller.py:40-197)
        for (int i = tid; i < N; i += NT) lub[i] = a.uWarm ? a.uWarm[slotU + i] : 0.0;
        bar();
        if (tid == 0 && fabs(lub[0]) < 2.220446049250313e-16) lub[0] = 2.220446049250313e-16;
        bar();
        EvalRes ev = PH(ph_evaluate)(c, nullptr, nullptr);
        double obj0 = ev.obj, mv0 = ev.maxv;
        const int maxScp = a.maxScp > 0 ? a.maxScp : P.maxScp;
        int qflags = 0, it = 0, status = SCPQP_ST_MAX_SCP;
        QpStats qs{0, 0, 0, 0};
        const bool warm_on = (P.flags & SCPQP_FLAG_COLD_QP) == 0;
        const int trStride = trace_stride(V, O, P.hpMax);
        bool prev_ok = false;   // previous QP certified: its active set seeds the next one
        for (it = 0; it < maxScp; ++it) {
#ifdef SCPQP_PROF
            _pt = __builtin_amdgcn_s_memtime();
#endif
            PH(ph_linearise)(c);
            PROF_ACC(11);
            // warm start from the previous QP's active set from the third QP on: the
            // first re-linearisation moves the active set too far for a few
            // active-set corrections to recover it (tools/polish_study.py: 0/16)
            const int ipm_before = qs.ipm, rounds_before = qs.rounds, refine_before = qs.refine;
            const bool warm_qp = warm_on && prev_ok && it >= 2;
            if constexpr (SH == 2) {   // c5: the QP with its horizon class compiled in
                if (Hb == 30) prev_ok = qp_solve<HG, VG, RM, OCC, 6>(c, &qflags, warm_qp, qs);
                else if (Hb == 20) prev_ok = qp_solve<HG, VG, RM, OCC, 5>(c, &qflags, warm_qp, qs);
                else if (Hb == 10) prev_ok = qp_solve<HG, VG, RM, OCC, 4>(c, &qflags, warm_qp, qs);
                else prev_ok = qp_solve<HG, VG, RM, OCC, SH>(c, &qflags, warm_qp, qs);
            } else {
                prev_ok = qp_solve<HG, VG, RM, OCC, SH>(c, &qflags, warm_qp, qs);
            }
#ifdef SCPQP_PROF
            _pt = __builtin_amdgcn_s_memtime();
#endif
            double* trp = (a.trace && it < P.maxScp) ? a.trace + ((size_t)b * P.maxScp + it) * trStride
                                                     : nullptr;
            if (trp) PH(ph_trace_rows)(c, trp);
            PH(ph_take_u)(c);
            ev = PH(ph_evaluate)(c, nullptr, nullptr);
            PROF_ACC(17);
            const double merit0 = obj0 + P.slackW * mv0;
            const double delta = merit0 - (ev.obj + P.slackW * ev.maxv);
            if (trp)
                PH(ph_trace_sol)(c, trp, D4{ev.obj, ev.maxv, ev.sumv, (double)ev.feasible}, delta,
                                 qs.ipm - ipm_before, (prev_ok ? 1 : 0) | (warm_qp ? 2 : 0), merit0,
                                 qs.rounds - rounds_before, qs.refine - refine_before);
            obj0 = ev.obj;
            mv0 = ev.maxv;
            if (!isfinite(ev.obj)) {
                status = SCPQP_ST_NUMERIC;
                break;
            }
            if (V == 1 && fabs(delta) < P.deltaTol && ev.maxv > P.ctol) {
                status = SCPQP_ST_CONVERGED;
                break;
            }
            if (fabs(delta) < P.deltaTol && ev.maxv <= P.ctol) {
                status = SCPQP_ST_CONVERGED;
                break;
            }
        }
        const int nscp = it < maxScp ? it + 1 : maxScp;
        if (V == 1 && !ev.feasible && status != SCPQP_ST_NUMERIC) status = SCPQP_ST_INVALID;
        // outputs (positions of the final u are in pb from the last evaluate)
        if (a.uOut)
            for (int i = tid; i < N; i += NT) a.uOut[slotU + i] = lub[i];
        if (a.trajOut)
            for (int i = tid; i < Hb * 2 * V; i += NT) {
                const int k = i / (2 * V), cc = (i / V) & 1, v = i % V;
                a.trajOut[(size_t)b * P.hpMax * 2 * V + i] = lpb[(v * Hb + k) * 2 + cc];
            }
        if (tid == 0) {
            if (a.status) a.status[b] = status | qflags | (sflag_any ? SCPQP_FL_SAMPLER : 0);
            if (a.nscp) a.nscp[b] = nscp;
            if (a.nipm) a.nipm[b] = qs.ipm;
            if (a.npol) a.npol[b] = qs.rounds;
            if (a.nref) a.nref[b] = qs.refine;
            if (a.nwarm) a.nwarm[b] = qs.warm_ok;
#ifdef SCPQP_PROF
            if (b < 8192) g_ptime[2 * b + 1] = __builtin_amdgcn_s_memrealtime();
#endif
            if (a.obj) a.obj[b] = ev.obj;
            if (a.maxv) a.maxv[b] = ev.maxv;
            if (a.sumv) a.sumv[b] = ev.sumv;
            if (a.feas) a.feas[b] = ev.feasible;
        }
        bar();
    }
}

}  // namespace

// ---------------------------------------------------------------------------
// Launch of one kernel instantiation.  csrc/kernels.hip instantiates these in groups,
// one translation unit per group (the library builds in parallel); the host side
// (scpqp.hip) declares them extern.  Returns a hipError_t.
// ---------------------------------------------------------------------------
namespace scpqp_kern {
template <bool HG, bool VG, int RM, int OCC, int SH>
int launch(const void* args, size_t lds, hipStream_t st, int grid) {
    auto kern = scp_kernel<HG, VG, RM, OCC, SH>;
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return (int)e;
    hipLaunchKernelGGL(kern, dim3(grid), dim3(NT), lds, st, *static_cast<const KArgs*>(args));
    return (int)hipGetLastError();
}

// Diagnostic counters of one translation unit's kernels (every unit has its own device
// globals; the host sums the units): what 0 = phase stamps (32), 1 = per-problem start /
// end times (2 n), 2 = the reduction-buffer check (2).  hipErrorInvalidValue when the
// build has no such counters.
template <int UNIT>
int diag_read(int what, unsigned long long* out, int n, int reset) {
    (void)out; (void)n; (void)reset;
#ifdef SCPQP_PROF
    if (what == 0) {
        hipError_t e = hipMemcpyFromSymbol(out, HIP_SYMBOL(g_prof), sizeof(unsigned long long) * 32);
        if (e == hipSuccess && reset) {
            unsigned long long z[32] = {0};
            e = hipMemcpyToSymbol(HIP_SYMBOL(g_prof), z, sizeof(z));
        }
        return (int)e;
    }
    if (what == 1)
        return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_ptime), sizeof(unsigned long long) * 2 * n);
#endif
#ifdef SCPQP_DIAG_REDUCE_CHECK
    if (what == 2) {
        unsigned v[2];
        hipError_t e = hipMemcpyFromSymbol(v, HIP_SYMBOL(g_redchk), sizeof(v));
        out[0] = v[0];
        out[1] = v[1];
        if (e == hipSuccess && reset) {
            const unsigned z[2] = {0, 0};
            e = hipMemcpyToSymbol(HIP_SYMBOL(g_redchk), z, sizeof(z));
        }
        return (int)e;
    }
#endif
    (void)what;
    return (int)hipErrorInvalidValue;
}
}  // namespace scpqp_kern
