// scpqp.hip — MI355X (gfx950) batched SCP-QP trajectory planner: the C-ABI of
// include/scpqp.h (host side).  The device code is in scpqp_kernel.h; its kernel
// instantiations are compiled in groups by kernels.hip (one translation unit per group,
// so the library builds in parallel) and declared extern below.

#include "scpqp_kernel.h"

#include <vector>

// Every kernel instantiation the dispatch (launch) can run: (HG, VG, RM, OCC, SH).
// kernels.hip instantiates each of them in exactly one group.
#define SCPQP_RT_LIST(X, HGV, VGV)                                                         \
    X(HGV, VGV, 1, 2, 0) X(HGV, VGV, 1, 3, 0) X(HGV, VGV, 2, 2, 0) X(HGV, VGV, 2, 3, 0)     \
    X(HGV, VGV, 3, 2, 0) X(HGV, VGV, 3, 3, 0) X(HGV, VGV, 4, 2, 0) X(HGV, VGV, 4, 3, 0)
#define SCPQP_KERNEL_LIST(X)                                                               \
    X(false, true, 2, 3, 1) X(true, true, 4, 2, 3) X(false, true, 2, 2, 2)                 \
    X(false, true, 2, 3, 2) X(true, true, 2, 3, 2)                                         \
    SCPQP_RT_LIST(X, true, true) SCPQP_RT_LIST(X, false, true) SCPQP_RT_LIST(X, false, false)
#define SCPQP_EXTERN_LAUNCH(HG, VG, RM, OCC, SH) \
    extern template int scpqp_kern::launch<HG, VG, RM, OCC, SH>(const void*, size_t, hipStream_t, int);
SCPQP_KERNEL_LIST(SCPQP_EXTERN_LAUNCH)
#ifdef SCPQP_DIAG
SCPQP_EXTERN_LAUNCH(false, true, 2, 4, 1)   // the OCC = 4 residency experiment (plan)
#endif
#undef SCPQP_EXTERN_LAUNCH
// kernels.hip's groups, each with its own diagnostic counters (diag_read<group>)
constexpr int kKernelGroups = 10;
extern template int scpqp_kern::diag_read<1>(int, unsigned long long*, int, int);
extern template int scpqp_kern::diag_read<2>(int, unsigned long long*, int, int);
extern template int scpqp_kern::diag_read<3>(int, unsigned long long*, int, int);
extern template int scpqp_kern::diag_read<4>(int, unsigned long long*, int, int);
extern template int scpqp_kern::diag_read<5>(int, unsigned long long*, int, int);
extern template int scpqp_kern::diag_read<6>(int, unsigned long long*, int, int);
extern template int scpqp_kern::diag_read<7>(int, unsigned long long*, int, int);
extern template int scpqp_kern::diag_read<8>(int, unsigned long long*, int, int);
extern template int scpqp_kern::diag_read<9>(int, unsigned long long*, int, int);
extern template int scpqp_kern::diag_read<10>(int, unsigned long long*, int, int);

namespace {

// ---------------------------------------------------------------------------
// Work order of a mixed-horizon batch (config c5): longest horizons first, so the
// expensive problems start at once and the cheap ones fill the tail (LPT list
// scheduling).  One workgroup: a counting sort of the problem indices by horizon,
// descending; horizons outside [1, hp_max] go last.  The order within a horizon is
// arbitrary (LDS atomics) and changes no result: every problem is solved on its own.
// ---------------------------------------------------------------------------
constexpr int kOrderThreads = 1024;
__global__ __launch_bounds__(kOrderThreads) void order_kernel(const int* hp, int B, int hpMax, int* perm) {
    __shared__ int cnt[SCPQP_MAX_HP + 2], off[SCPQP_MAX_HP + 2];
    const int tid = threadIdx.x;
    auto bucket = [&](int b) {
        const int h = hp[b];
        return (h >= 1 && h <= hpMax) ? h : 0;
    };
    for (int h = tid; h < SCPQP_MAX_HP + 2; h += kOrderThreads) cnt[h] = 0;
    __syncthreads();
    for (int b = tid; b < B; b += kOrderThreads) atomicAdd(&cnt[bucket(b)], 1);
    __syncthreads();
    if (tid == 0) {
        int start = 0;
        for (int h = hpMax; h >= 1; --h) {
            off[h] = start;
            start += cnt[h];
        }
        off[0] = start;
    }
    __syncthreads();
    for (int b = tid; b < B; b += kOrderThreads) perm[atomicAdd(&off[bucket(b)], 1)] = b;
}

thread_local char g_err[512] = "";

int fail(int code, const char* fmt, const char* detail = "") {
    snprintf(g_err, sizeof(g_err), fmt, detail);
    return code;
}

#define HIPCHK(x)                                                                          \
    do {                                                                                   \
        hipError_t e_ = (x);                                                               \
        if (e_ != hipSuccess) return fail(SCPQP_E_HIP, "HIP error: %s", hipGetErrorString(e_)); \
    } while (0)

}  // namespace

struct scpqp_handle {
    scpqp_dims dims;
    DevParams hostP;
    DevParams* devP = nullptr;
    int device = 0;
    int cus = 256;
    int* counter = nullptr;
    int* perm = nullptr;   // work order of mixed-horizon solves (order_kernel), max_batch ints
    double* ws = nullptr;
    size_t wsBytes = 0;
    int hG = 0, vG = 0, occ = 2;
    size_t ldsBytes = 0;
    long long wsStride = 0;
    int grid = 0;
};

namespace {

const size_t kLdsLimit = 163840;
const size_t kLdsGranule = 2048;
// workgroups per CU at three waves per SIMD (the 168-VGPR budget of OCC = 3)
const int kMaxPerCU = 12 / NWAVE;

int plan(scpqp_handle* h) {
    const int V = h->dims.n_veh, O = h->dims.n_obst, Hm = h->dims.hp_max;
    // Plans: 0 everything in LDS, 1 constraint vectors in the workspace (lean at two
    // workgroups per CU: W~ and the constraint rows too), 2 also the KKT matrix.  The
    // register budget is compiled for 2 or 3 workgroups per CU (OCC), and the device
    // runs plan 1 lean exactly when OCC = 2 (Lay::LEAN).  A plan with the factor in LDS
    // is taken whenever it fits two workgroups per CU: its panel chain and trailing
    // update run on LDS latencies, and with the factor in the workspace a problem is
    // ~2.7x slower (4 vehicles at Hp 30: profiles/r03_c5_classes.txt); among the rest,
    // the most workgroups per CU (the kernel is latency-bound), then less in global
    // memory.
#ifdef SCPQP_DIAG
    const char* force = getenv("SCPQP_PLAN");   // diagnostic build: force a plan
#else
    const char* force = nullptr;
#endif
    const int cfg0 = force ? atoi(force) : 0, cfg1 = force ? cfg0 + 1 : 3;
    int best = -1, bestPer = 0, bestKey = -1;
    bool bestLean = false;
    for (int cfg = cfg0; cfg < cfg1 && cfg < 3; ++cfg) {
        for (int ln = 0; ln < (cfg == 1 ? 2 : 1); ++ln) {
            const bool lean = ln == 1;
            const Off f = plan_offsets(V, O, Hm, cfg >= 2, cfg >= 1, lean);
            const size_t lds = (size_t)(f.persist + f.uni) * sizeof(double);
            if (lds > kLdsLimit) continue;
            // residency at the LDS allocation granularity: a c2 plan of 53,888 B (3 x 161,664 B
            // by byte count) ran as if fewer than three workgroups fit per CU (round 6,
            // profiles/r06_ab_tv_lds.txt); 2 KB granules agree with every plan measured
            int perCU = (int)(kLdsLimit / ((lds + kLdsGranule - 1) / kLdsGranule * kLdsGranule));
            // beyond 3 waves per SIMD the register budget, not LDS, bounds residency
            if (perCU > kMaxPerCU) perCU = kMaxPerCU;
            if (cfg == 1 && !lean && perCU < 3) continue;   // OCC 2 runs plan 1 lean
            if (lean && perCU > 2) perCU = 2;
            const int key = ((cfg < 2 && perCU >= 2) ? 1000 : 0) + 10 * perCU + (2 - cfg);
            if (key > bestKey) {
                best = cfg;
                bestPer = perCU;
                bestKey = key;
                bestLean = lean;
            }
        }
    }
#ifdef SCPQP_DIAG
    // diagnostic build: SCPQP_OCC4=1 runs the lean plan 1 at four workgroups per CU (the
    // 128-VGPR budget of OCC = 4) when it fits (the round-6 c2 residency experiment)
    if (const char* o4 = getenv("SCPQP_OCC4")) {
        const Off f = plan_offsets(V, O, Hm, false, true, true);
        if (atoi(o4) == 1 && (size_t)(f.persist + f.uni) * sizeof(double) * 4 <= kLdsLimit) {
            h->hG = 0;
            h->vG = 1;
            h->ldsBytes = (size_t)(f.persist + f.uni) * sizeof(double);
            h->wsStride = f.ws;
            h->grid = h->cus * 4;
            h->occ = 4;
            return 0;
        }
    }
#endif
    if (best < 0) return fail(SCPQP_E_SIZE, "problem too large for the LDS plan%s");
    const Off f = plan_offsets(V, O, Hm, best >= 2, best >= 1, bestLean);
    h->hG = best >= 2;
    h->vG = best >= 1;
    h->ldsBytes = (size_t)(f.persist + f.uni) * sizeof(double);
    h->wsStride = f.ws;
    h->grid = h->cus * bestPer;
    // waves per SIMD the register budget is compiled for (template OCC)
    h->occ = (bestPer * NWAVE + 3) / 4 >= 3 ? 3 : 2;
    return 0;
}

typedef int (*KernelLaunch)(const void*, size_t, hipStream_t, int);
int run_kernel(KernelLaunch fn, scpqp_handle* h, const KArgs& a, hipStream_t st, int grid) {
    const int e = fn(&a, h->ldsBytes, st, grid);
    if (e != 0) return fail(SCPQP_E_HIP, "HIP error: %s", hipGetErrorString(static_cast<hipError_t>(e)));
    return 0;
}
#define SCPQP_RUN(HG, VG, RM, OCC, SH) run_kernel(scpqp_kern::launch<HG, VG, RM, OCC, SH>, h, a, st, grid)

// the kernel groups' diagnostic counters, summed (diag_read)
int diag_sum(int what, unsigned long long* out, int count, int n, int reset) {
    typedef int (*DiagRead)(int, unsigned long long*, int, int);
    static const DiagRead units[kKernelGroups] = {
        scpqp_kern::diag_read<1>, scpqp_kern::diag_read<2>, scpqp_kern::diag_read<3>,
        scpqp_kern::diag_read<4>, scpqp_kern::diag_read<5>, scpqp_kern::diag_read<6>,
        scpqp_kern::diag_read<7>, scpqp_kern::diag_read<8>, scpqp_kern::diag_read<9>,
        scpqp_kern::diag_read<10>};
    std::vector<unsigned long long> part(count);
    for (int i = 0; i < count; ++i) out[i] = 0;
    for (int u = 0; u < kKernelGroups; ++u) {
        const int e = units[u](what, part.data(), n, reset);
        if (e != 0) return fail(SCPQP_E_HIP, "HIP error: %s", hipGetErrorString(static_cast<hipError_t>(e)));
        for (int i = 0; i < count; ++i) out[i] += part[i];
    }
    return 0;
}

int launch(scpqp_handle* h, KArgs& a, hipStream_t st) {
    if (a.B <= 0) return 0;
    HIPCHK(hipSetDevice(h->device));
    int grid = a.B < h->grid ? a.B : h->grid;
#ifdef SCPQP_DIAG
    if (const char* g = getenv("SCPQP_GRID")) {   // diagnostic build: fewer resident workgroups
        const int cap = atoi(g);
        if (cap > 0 && cap < grid) grid = cap;
    }
#endif
    if (h->wsStride > 0) {
        const size_t need = (size_t)grid * h->wsStride * sizeof(double);
        if (need > h->wsBytes) {
            if (h->ws) HIPCHK(hipFree(h->ws));
            h->ws = nullptr;
            HIPCHK(hipMalloc(&h->ws, need));
            h->wsBytes = need;
        }
    }
    a.P = h->devP;
    a.ws = h->ws;
    a.wsStride = h->wsStride;
    a.counter = h->counter;
    HIPCHK(hipMemsetAsync(h->counter, 0, sizeof(int), st));
    a.perm = nullptr;
#ifdef SCPQP_DIAG
    const char* ord = getenv("SCPQP_ORDER");   // diagnostic build: SCPQP_ORDER=0 keeps the input order
    const bool keep_order = ord && atoi(ord) == 0;
#else
    const bool keep_order = false;
#endif
    if (a.mode == MODE_SOLVE && a.hp && h->perm && !keep_order) {
        hipLaunchKernelGGL(order_kernel, dim3(1), dim3(kOrderThreads), 0, st, a.hp, a.B, h->dims.hp_max,
                           h->perm);
        HIPCHK(hipGetLastError());
        a.perm = h->perm;
    }
    const int R = (h->dims.n_veh * h->dims.hp_max + 1 + 63) / 64;   // row slots of the solves
    const int occ = h->occ;   // waves per SIMD the register budget is compiled for
    // compile-time shapes (shape_c): the BASELINE configurations' instantiations
    const scpqp_dims& d = h->dims;
    int sh = 0;
    if (d.n_obst == 0 && d.n_veh == 4) sh = (d.hp_max == 20 && !a.hp) ? 1 : 2;
    if (d.n_obst == 0 && d.n_veh == 8 && d.hp_max == 30 && !a.hp) sh = 3;
#ifdef SCPQP_DIAG
    if (const char* e = getenv("SCPQP_SHAPE"))   // diagnostic build: SCPQP_SHAPE=0 runs the runtime shape
        if (atoi(e) == 0) sh = 0;
#endif
    if (sh == 1 && !h->hG && h->vG && R == 2 && occ == 3) return SCPQP_RUN(false, true, 2, 3, 1);
#ifdef SCPQP_DIAG
    if (sh == 1 && !h->hG && h->vG && R == 2 && occ == 4) return SCPQP_RUN(false, true, 2, 4, 1);
#endif
    if (sh == 2 && h->vG && R == 2 && occ == 3) {
        if (h->hG) return SCPQP_RUN(true, true, 2, 3, 2);
        return SCPQP_RUN(false, true, 2, 3, 2);
    }
    if (sh == 2 && !h->hG && h->vG && R == 2 && occ == 2) return SCPQP_RUN(false, true, 2, 2, 2);
    if (sh == 3 && h->hG && R == 4 && occ == 2) return SCPQP_RUN(true, true, 4, 2, 3);
#define SCPQP_DISPATCH(HGV, VGV)                                              \
    switch (R * 4 + occ) {                                                   \
        case 6: return SCPQP_RUN(HGV, VGV, 1, 2, 0);          \
        case 7: return SCPQP_RUN(HGV, VGV, 1, 3, 0);          \
        case 10: return SCPQP_RUN(HGV, VGV, 2, 2, 0);         \
        case 11: return SCPQP_RUN(HGV, VGV, 2, 3, 0);         \
        case 14: return SCPQP_RUN(HGV, VGV, 3, 2, 0);         \
        case 15: return SCPQP_RUN(HGV, VGV, 3, 3, 0);         \
        case 19: return SCPQP_RUN(HGV, VGV, 4, 3, 0);         \
        default: return SCPQP_RUN(HGV, VGV, 4, 2, 0);         \
    }
    if (h->hG) { SCPQP_DISPATCH(true, true) }
    if (h->vG) { SCPQP_DISPATCH(false, true) }
    SCPQP_DISPATCH(false, false)
#undef SCPQP_DISPATCH
}

// need_obst: the entry point reads the obstacle predictions (solve, evaluate);
// MPCclass linearisation and reference sampling do not (MPC_Iter.py:59-149).
int check_in(scpqp_handle* h, int32_t B, const scpqp_batch_in* in, bool need_obst) {
    if (!h) return fail(SCPQP_E_ARG, "null handle%s");
    if (!in) return fail(SCPQP_E_ARG, "null input struct%s");
    if (B < 0 || B > h->dims.max_batch) return fail(SCPQP_E_ARG, "batch size out of range%s");
    if (B == 0) return 0;   // empty batch: no launch, buffers may be null
    if (!in->x0) return fail(SCPQP_E_ARG, "null input x0%s");
    if (need_obst && h->dims.n_obst > 0 && !in->obst)
        return fail(SCPQP_E_ARG, "n_obst > 0 needs obst%s");
    return 0;
}

KArgs base_args(int32_t B, const scpqp_batch_in* in) {
    KArgs a;
    memset(&a, 0, sizeof(a));
    a.B = B;
    a.x0 = in->x0;
    a.u0 = in->u0;
    a.ec = in->ec_noise;
    a.obst = in->obst;
    a.refIn = in->ref_points;
    a.uWarm = in->u_warm;
    a.hp = in->hp;
    a.maxScp = in->max_scp_iter;
    return a;
}

}  // namespace

// error reporting for the other translation units of the library (plant.hip)
int scpqp_fail_(int code, const char* msg) { return fail(code, "%s", msg); }

extern "C" {

const char* scpqp_last_error(void) { return g_err; }

const char* scpqp_version(void) { return "scpqp-mi355x 0.4 (gfx950, fp64)"; }

int scpqp_create(const scpqp_dims* dims, const scpqp_params* p, int device, scpqp_handle** out) {
    if (!dims || !p || !out) return fail(SCPQP_E_ARG, "null argument%s");
    *out = nullptr;
    if (dims->n_veh < 1 || dims->n_veh > SCPQP_MAX_VEH) return fail(SCPQP_E_ARG, "n_veh out of range%s");
    if (dims->n_obst < 0 || dims->n_obst > SCPQP_MAX_OBST) return fail(SCPQP_E_ARG, "n_obst out of range%s");
    if (dims->hp_max < 1 || dims->hp_max > SCPQP_MAX_HP) return fail(SCPQP_E_ARG, "hp_max out of range%s");
    if (dims->n_veh * dims->hp_max + 1 > 256) return fail(SCPQP_E_SIZE, "n_veh*hp_max+1 > 256%s");
    if (dims->max_batch < 0) return fail(SCPQP_E_ARG, "max_batch < 0%s");
    if (!p->lf || !p->lr || !p->q || !p->q_final || !p->r || !p->dsafe_veh)
        return fail(SCPQP_E_ARG, "null per-vehicle parameter%s");
    if (dims->n_obst > 0 && !p->dsafe_obs) return fail(SCPQP_E_ARG, "n_obst > 0 needs dsafe_obs%s");
    if (p->ref_max_pts > SCPQP_MAX_REFPTS) return fail(SCPQP_E_ARG, "ref_max_pts too large%s");
    scpqp_handle* h = new (std::nothrow) scpqp_handle();
    if (!h) return fail(SCPQP_E_NOMEM, "out of host memory%s");
    h->dims = *dims;
    h->device = device;
    DevParams& P = h->hostP;
    memset(&P, 0, sizeof(P));
    const int V = dims->n_veh, O = dims->n_obst;
    P.nV = V;
    P.hpMax = dims->hp_max;
    P.nO = O;
    P.maxPts = p->ref_max_pts > 0 ? p->ref_max_pts : 2;
    P.maxScp = p->max_scp_iter > 0 ? p->max_scp_iter : 20;
    P.maxIpm = p->max_ipm_iter > 0 ? p->max_ipm_iter : 60;
    P.nRefine = p->polish_refine > 0 ? p->polish_refine : 40;
    P.flags = p->flags;
    P.dt = p->dt;
    P.uLim = p->u_lim;
    P.ctol = p->constraint_tol;
    P.deltaTol = p->delta_tol;
    P.slackW = p->slack_weight;
    P.ipmTol = p->ipm_tol > 0 ? p->ipm_tol : 1e-9;
    P.polDelta = p->polish_delta > 0 ? p->polish_delta : 3e-7;
    P.polRho = p->polish_rho >= 0 ? p->polish_rho : 1e-12;
    for (int v = 0; v < V; ++v) {
        P.Lf[v] = p->lf[v];
        P.Lr[v] = p->lr[v];
        P.Q[v] = p->q[v];
        P.Qf[v] = p->q_final[v];
        P.R[v] = p->r[v];
        for (int w = 0; w < V; ++w) {
            const double ds = p->dsafe_veh[v * V + w] + p->dsafe_extra;
            P.D2veh[v * SCPQP_MAX_VEH + w] = ds * ds;
        }
        for (int o = 0; o < O; ++o) {
            const double ds = p->dsafe_obs[v * O + o] + p->dsafe_extra;
            P.D2obs[v * SCPQP_MAX_OBST + o] = ds * ds;
        }
        const int np = p->ref_npts ? p->ref_npts[v] : 0;
        P.npts[v] = np;
        for (int i = 0; i < np && p->ref_polyline; ++i) {
            P.poly[(v * P.maxPts + i) * 2] = p->ref_polyline[(v * p->ref_max_pts + i) * 2];
            P.poly[(v * P.maxPts + i) * 2 + 1] = p->ref_polyline[(v * p->ref_max_pts + i) * 2 + 1];
        }
    }
    hipError_t e = hipSetDevice(device);
    if (e == hipSuccess) e = hipDeviceGetAttribute(&h->cus, hipDeviceAttributeMultiprocessorCount, device);
    if (e == hipSuccess) e = hipMalloc(&h->devP, sizeof(DevParams));
    if (e == hipSuccess) e = hipMemcpy(h->devP, &P, sizeof(DevParams), hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMalloc(&h->counter, sizeof(int));
    if (e == hipSuccess && dims->max_batch > 0)
        e = hipMalloc(&h->perm, sizeof(int) * (size_t)dims->max_batch);
    if (e != hipSuccess) {
        snprintf(g_err, sizeof(g_err), "HIP error: %s", hipGetErrorString(e));
        scpqp_destroy(h);
        return SCPQP_E_HIP;
    }
    const int rc = plan(h);
    if (rc) {
        scpqp_destroy(h);
        return rc;
    }
    *out = h;
    return 0;
}

int scpqp_destroy(scpqp_handle* h) {
    if (!h) return 0;
    (void)hipSetDevice(h->device);
    if (h->devP) (void)hipFree(h->devP);
    if (h->counter) (void)hipFree(h->counter);
    if (h->perm) (void)hipFree(h->perm);
    if (h->ws) (void)hipFree(h->ws);
    delete h;
    return 0;
}

int scpqp_solve(scpqp_handle* h, int32_t B, const scpqp_batch_in* in, const scpqp_batch_out* out,
                void* stream) {
    const int rc = check_in(h, B, in, true);
    if (rc) return rc;
    if (!out) return fail(SCPQP_E_ARG, "null output struct%s");
    KArgs a = base_args(B, in);
    a.mode = MODE_SOLVE;
    a.uOut = out->u;
    a.trajOut = out->traj;
    a.status = out->status;
    a.nscp = out->n_scp;
    a.nipm = out->n_ipm;
    a.obj = out->obj;
    a.maxv = out->max_violation;
    a.sumv = out->sum_violations;
    a.feas = out->feasible;
    a.npol = out->n_polish;
    a.nref = out->n_refine;
    a.nwarm = out->n_warm;
    a.trace = out->trace;
    return launch(h, a, static_cast<hipStream_t>(stream));
}

int scpqp_linearize(scpqp_handle* h, int32_t B, const scpqp_batch_in* in, const scpqp_lin_out* out,
                    void* stream) {
    const int rc = check_in(h, B, in, false);
    if (rc) return rc;
    if (!out) return fail(SCPQP_E_ARG, "null output struct%s");
    KArgs a = base_args(B, in);
    a.mode = MODE_LINEARIZE;
    a.Ad = out->Ad;
    a.Bd = out->Bd;
    a.Ed = out->Ed;
    a.gOut = out->g;
    a.p0Out = out->const_term;
    a.psiOut = out->psi0;
    a.refOut = out->ref_points;
    return launch(h, a, static_cast<hipStream_t>(stream));
}

int scpqp_evaluate(scpqp_handle* h, int32_t B, const scpqp_batch_in* in, const double* u,
                   const scpqp_eval_out* out, void* stream) {
    const int rc = check_in(h, B, in, true);
    if (rc) return rc;
    if (B == 0) return 0;
    if (!out || !u) return fail(SCPQP_E_ARG, "null u or output struct%s");
    KArgs a = base_args(B, in);
    a.mode = MODE_EVALUATE;
    a.uEval = u;
    a.obj = out->obj;
    a.maxv = out->max_violation;
    a.sumv = out->sum_violations;
    a.feas = out->feasible;
    a.cveh = out->c_veh;
    a.cobs = out->c_obs;
    a.trajOut = out->traj;
    return launch(h, a, static_cast<hipStream_t>(stream));
}

int scpqp_sample_reference(scpqp_handle* h, int32_t B, const scpqp_batch_in* in, double* ref,
                           void* stream) {
    const int rc = check_in(h, B, in, false);
    if (rc) return rc;
    if (B == 0) return 0;
    if (!ref) return fail(SCPQP_E_ARG, "null ref_points%s");
    KArgs a = base_args(B, in);
    a.refIn = nullptr;
    a.mode = MODE_SAMPLE;
    a.refOut = ref;
    return launch(h, a, static_cast<hipStream_t>(stream));
}

#ifdef SCPQP_PROF
int scpqp_prof_times(unsigned long long* out, int n) { return diag_sum(1, out, 2 * n, n, 0); }
int scpqp_prof_read(unsigned long long* out, int reset) { return diag_sum(0, out, 32, 0, reset); }
#endif
#ifdef SCPQP_DIAG_REDUCE_CHECK
// {block reductions run, reductions that reused the previous reduction's buffer with no
// barrier between them} since the last reset (must be 0), over every kernel group
int scpqp_diag_reduce_check(unsigned long long* out, int reset) { return diag_sum(2, out, 2, 0, reset); }
#endif

int scpqp_trace_layout(scpqp_handle* h, int32_t* stride, int32_t* iters) {
    if (!h) return fail(SCPQP_E_ARG, "null handle%s");
    if (stride) *stride = trace_stride(h->dims.n_veh, h->dims.n_obst, h->dims.hp_max);
    if (iters) *iters = h->hostP.maxScp;
    return 0;
}

int scpqp_resources(scpqp_handle* h, int64_t* lds, int64_t* ws, int32_t* big, int32_t* grid) {
    if (!h) return fail(SCPQP_E_ARG, "null handle%s");
    if (lds) *lds = (int64_t)h->ldsBytes;
    if (ws) *ws = (int64_t)h->wsStride * (int64_t)sizeof(double);
    if (big) *big = h->hG ? 2 : (h->vG ? 1 : 0);
    if (grid) *grid = h->grid;
    return 0;
}

}  // extern "C"
