/*
 * scpqp.h — C-ABI of the MI355X batched SCP-QP trajectory planner.
 *
 * Drop-in boundary for the hot path of Zhang-Xiaoxue/Senquential-Convex-
 * Programming-for-Trajectory-Planning.  The reference's boundary is an
 * in-process Python class API:
 *
 *   SCPcontroller(scenario, Iter, prevOutput)          SCP_controller.py:18-38
 *   .SCP_controller(Iter) -> (U, traj, out)             SCP_controller.py:40-72
 *   .QCQP_evaluate(U)     -> 8-tuple                    SCP_controller.py:215-265
 *   MPCclass(scenario, Iter)                            MPC_Iter.py:57-149
 *   sampleReferenceTrajectory(...)                      SampleReferTraj.py:8-32
 *
 * Each entry point below replaces one of those for a whole BATCH of problems
 * (one problem = one joint multi-vehicle QCQP of one MPC step).  The Python
 * drop-in modules (SCP_controller.py, MPC_Iter.py, ... in the package
 * directory) bind these through ctypes; see INTEGRATION.md.
 *
 * Conventions
 *   - every array argument is a caller-owned DEVICE pointer (e.g. a torch-ROCm
 *     tensor's data_ptr), float64 / int32, C-contiguous, problem-major;
 *   - per-problem arrays are laid out in the reference's own layout for that
 *     problem's horizon hp_b (<= hp_max), inside a slot sized for hp_max;
 *   - calls are asynchronous on `stream` (a hipStream_t; NULL = default);
 *   - return 0 on success, a negative SCPQP_E* code on an API error (message
 *     in scpqp_last_error(), thread-local).  Numerical trouble in one problem
 *     never aborts the batch: it is reported in that problem's status word.
 *   - one handle per host thread; the handle owns its device workspace.
 */
#ifndef SCPQP_H
#define SCPQP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SCPQP_MAX_VEH 16
#define SCPQP_MAX_OBST 32
#define SCPQP_MAX_REFPTS 8
#define SCPQP_MAX_HP 64

#define SCPQP_OK 0
#define SCPQP_E_ARG -1
#define SCPQP_E_HIP -2
#define SCPQP_E_NOMEM -3
#define SCPQP_E_SIZE -4

/* per-problem status word (scpqp_batch_out.status) */
#define SCPQP_ST_CONVERGED 0        /* stopping rule met, SCP_controller.py:191-195  */
#define SCPQP_ST_MAX_SCP 1          /* 20 QPs without meeting it (SCP_controller.py:92) */
#define SCPQP_ST_INVALID 2          /* nVeh==1 and infeasible: controllerOutput['resultInvalid'] */
#define SCPQP_ST_NUMERIC 3          /* non-finite iterate */
#define SCPQP_FL_POLISH_REJECTED 0x100   /* some QP kept the IPM iterate (polish not certified) */
#define SCPQP_FL_IPM_MAXIT 0x200         /* some QP hit the IPM iteration cap                 */
#define SCPQP_FL_SAMPLER 0x400           /* reference sampler left its documented domain (B.2) */

/* scenario-level sizes (SCP_controller.py:27-31, MPC_Iter.py:66-72) */
typedef struct scpqp_dims {
    int32_t n_veh;       /* scenario.nVeh                               */
    int32_t hp_max;      /* largest prediction horizon (Hu == Hp)       */
    int32_t n_obst;      /* scenario.nObst                              */
    int32_t max_batch;   /* largest B passed to any call on this handle */
} scpqp_dims;

/* scenario-level parameters; every pointer is a HOST pointer, copied at create */
typedef struct scpqp_params {
    double dt;               /* scenario.dt after complete_scenario (Scenarios.py:207) */
    double u_lim;            /* scenario.uLim (SCP_controller.py:34, build choice B.7) */
    double dsafe_extra;      /* scenario.dsafeExtra (Scenarios.py:58)                  */
    double constraint_tol;   /* Config.QCQP.constraintTolerance = 4.2e-3 (Config.py:18)*/
    double delta_tol;        /* 1e-3 (SCP_controller.py:83)                            */
    double slack_weight;     /* 1e5  (SCP_controller.py:84)                            */
    int32_t max_scp_iter;    /* 20   (SCP_controller.py:86)                            */
    int32_t max_ipm_iter;    /* IPM iteration cap per QP (e.g. 60)                     */
    int32_t polish_refine;   /* cap on multiplier-iteration solves per round (0: 40) */
    int32_t flags;           /* SCPQP_FLAG_* (obstacle quirk B.4 on by default)        */
    double ipm_tol;          /* scaled KKT tolerance of the IPM (e.g. 1e-9)            */
    double polish_delta;     /* polish penalty delta (scaled units, default 3e-7)      */
    double polish_rho;       /* polish proximal rho (e.g. 1e-12)                       */
    const double* lf;        /* [n_veh] scenario.Lf                                    */
    const double* lr;        /* [n_veh] scenario.Lr                                    */
    const double* q;         /* [n_veh] scenario.Q                                     */
    const double* q_final;   /* [n_veh] scenario.Q_final                               */
    const double* r;         /* [n_veh] scenario.R                                     */
    const double* dsafe_veh; /* [n_veh*n_veh] scenario.dsafeVehicles                   */
    const double* dsafe_obs; /* [n_veh*n_obst] scenario.dsafeObstacles (NULL if none)  */
    const double* ref_polyline; /* [n_veh][ref_max_pts][2] scenario.referenceTrajectories */
    const int32_t* ref_npts; /* [n_veh] points per polyline (>= 2)                     */
    int32_t ref_max_pts;
} scpqp_params;

#define SCPQP_FLAG_OBST_QUIRK 1   /* evaluate obstacles inside the v2 loop    */
#define SCPQP_FLAG_COLD_QP 2      /* no active-set warm start between SCP iterations       */

/* per-call inputs (DEVICE pointers) */
typedef struct scpqp_batch_in {
    const double* x0;        /* [B][n_veh][6]   Iter.x0                                */
    const double* u0;        /* [B][n_veh]      Iter.u0                                */
    const double* ec_noise;  /* [B][n_veh][2]   Model.py:85-86 draws, or NULL (no noise)*/
    const int32_t* hp;       /* [B]             per-problem horizon, or NULL (= hp_max)*/
    const double* obst;      /* [B][n_obst][2][hp_b]  Iter.obstacleFutureTrajectories  */
    const double* ref_points;/* [B][hp_b][2][n_veh]   Iter.ReferenceTrajectoryPoints,
                                or NULL: sampled on the device from the polylines      */
    const double* u_warm;    /* [B][n_veh*hp_b] prevOutput['u'] (vehicle-major), or NULL*/
    int32_t max_scp_iter;    /* 0: handle default; else override (e.g. 1 = one QP)     */
    int32_t reserved;
} scpqp_batch_in;

/* per-call outputs of scpqp_solve (DEVICE pointers; any may be NULL) */
typedef struct scpqp_batch_out {
    double* u;               /* [B][n_veh*hp_b]   controllerOutput['u']                */
    double* traj;            /* [B][hp_b][2][n_veh] trajectoryPrediction               */
    int32_t* status;         /* [B] SCPQP_ST_* | SCPQP_FL_*                            */
    int32_t* n_scp;          /* [B] QPs solved                                         */
    int32_t* n_ipm;          /* [B] IPM iterations summed over the QPs                 */
    double* obj;             /* [B] QCQP objective of the returned u                   */
    double* max_violation;   /* [B]                                                    */
    double* sum_violations;  /* [B]                                                    */
    int32_t* feasible;       /* [B]                                                    */
    int32_t* n_polish;       /* [B] active-set polish rounds summed over the QPs       */
    int32_t* n_refine;       /* [B] multiplier-iteration solves summed over the QPs    */
    int32_t* n_warm;         /* [B] QPs certified from the previous QP's active set    */
    double* trace;           /* [B][trace_iters][trace_stride] per-SCP-iteration record
                                (SCP_controller.py:169-189 optimization_log), or NULL.
                                Layout of one iteration (doubles), see scpqp_trace_layout:
                                  [0] delta  [1] obj  [2] max_violation  [3] sum_violations
                                  [4] slack omega = z[N]  [5] IPM iterations of this QP
                                  [6] QP flags (1 certified, 2 warm-started)  [7] feasible
                                  [8] obj_0 + 1e5 max_violation_0, the merit before this
                                      iteration (delta_hat = [8] - fval, :159)
                                  [9] this QP's polish rounds + 4096 x its polish solves
                                  [10, 10+N)        u_lin: the iterate the rows linearise at
                                  [10+N, 10+2N)     u: this QP's solution z[:N]
                                  [10+2N, 10+2N+4m) rows r: e_r[0], e_r[1], w_r, h_r (scaled
                                                  factored row); Aineq/bineq
                                                  follow as A_r = -(e_r.g) nrm/uLim,
                                                  b_r = h_r nrm, nrm = -1/w_r
                                N = n_veh*hp_max, m = pair + obstacle rows at hp_max;
                                a problem of horizon hp_b fills the prefixes of each part
                                (N_b = n_veh*hp_b, m_b rows).  Iterations past
                                trace_iters are not recorded.                          */
} scpqp_batch_out;

/* outputs of scpqp_linearize (MPCclass intermediates; DEVICE pointers, any may be NULL) */
typedef struct scpqp_lin_out {
    double* Ad;              /* [B][n_veh][6][6]                                       */
    double* Bd;              /* [B][n_veh][6]                                          */
    double* Ed;              /* [B][n_veh][6]                                          */
    double* g;               /* [B][n_veh][hp_b][2]  g_m = C A^m B (Mathcal_B blocks)   */
    double* const_term;      /* [B][n_veh][hp_b][2]  MPCclass.const_term               */
    double* psi0;            /* [B][n_veh][hp_b]     MPCclass.Psi_0                    */
    double* ref_points;      /* [B][hp_b][2][n_veh]                                    */
} scpqp_lin_out;

/* outputs of scpqp_evaluate (QCQP_evaluate; DEVICE pointers, any may be NULL) */
typedef struct scpqp_eval_out {
    double* obj;             /* [B] objValue                                           */
    double* max_violation;   /* [B]                                                    */
    double* sum_violations;  /* [B]                                                    */
    int32_t* feasible;       /* [B]                                                    */
    double* c_veh;           /* [B][n_veh][n_veh][hp_b] constraintValuesVehicle (-inf unset) */
    double* c_obs;           /* [B][n_veh][n_obst][hp_b] constraintValuesObstacle      */
    double* traj;            /* [B][hp_b][2][n_veh] forward_U trajectory (SCP_controller.py:199-213) */
} scpqp_eval_out;

typedef struct scpqp_handle scpqp_handle;

/* Replaces SCPcontroller construction-time state (SCP_controller.py:19-38). */
int scpqp_create(const scpqp_dims* dims, const scpqp_params* params, int device,
                 scpqp_handle** out);
int scpqp_destroy(scpqp_handle* h);
const char* scpqp_last_error(void);
const char* scpqp_version(void);

/* SCPcontroller.SCP_controller for B problems (SCP_controller.py:40-197):
 * MPCclass linearisation, constraint linearisation, QP loop, forward_U. */
int scpqp_solve(scpqp_handle* h, int32_t B, const scpqp_batch_in* in,
                const scpqp_batch_out* out, void* stream);

/* MPCclass(scenario, Iter) for B problems (MPC_Iter.py:59-149). */
int scpqp_linearize(scpqp_handle* h, int32_t B, const scpqp_batch_in* in,
                    const scpqp_lin_out* out, void* stream);

/* SCPcontroller.QCQP_evaluate(U) + forward_U(U) for B problems
 * (SCP_controller.py:199-265); u: [B][n_veh*hp_b] device. */
int scpqp_evaluate(scpqp_handle* h, int32_t B, const scpqp_batch_in* in, const double* u,
                   const scpqp_eval_out* out, void* stream);

/* sampleReferenceTrajectory for every vehicle of B problems (SampleReferTraj.py:8-32,
 * called as MPC_Iter.py:36-43); ref_points: [B][hp_b][2][n_veh] device. */
int scpqp_sample_reference(scpqp_handle* h, int32_t B, const scpqp_batch_in* in,
                           double* ref_points, void* stream);

/* Bytes of dynamic LDS and global workspace per workgroup the solve kernel
 * uses for this handle (diagnostics / roofline bookkeeping). */
int scpqp_resources(scpqp_handle* h, int64_t* lds_bytes, int64_t* ws_bytes_per_wg,
                    int32_t* big_mode, int32_t* grid);

/* Shape of scpqp_batch_out.trace for this handle: doubles per iteration and
 * iterations per problem (= the handle's max_scp_iter). */
int scpqp_trace_layout(scpqp_handle* h, int32_t* stride_doubles, int32_t* iters);

/* ------------------------------------------------------------------------
 * The bicycle plant around the solve (csrc/plant.hip).  Handle-free; every
 * array is a DEVICE pointer (float64, C-contiguous), calls are asynchronous
 * on `stream`.  The reference integrates with scipy odeint / dopri5; these
 * use fixed-step RK4 with steps of at most h_max seconds (2.5e-3 recommended:
 * ~1e-11 from the exact flow, below the reference's 1e-8 tolerances).
 * ---------------------------------------------------------------------- */
typedef struct scpqp_plant_params {
    int32_t n_veh;                 /* scenario.nVeh                       */
    int32_t pad0;
    double lf[SCPQP_MAX_VEH];      /* scenario.Lf (Model.py:26)           */
    double lr[SCPQP_MAX_VEH];      /* scenario.Lr (Model.py:27)           */
} scpqp_plant_params;

/* IterClass delay compensation (MPC_Iter.py:24-33): integrate Model.ode from
 * x_meas [B][n_veh][6] over linspace(0, horizon, n_out) with the constant
 * steering command u_hold [B][n_veh] (= u_path[v, -1]).  noise [B][n_veh][2]
 * (may be NULL): constant additive terms of dx[0], dx[1] (Model.py:84-86).
 * x0_out [B][n_veh][6] = Y[-1]; traj_out [B][n_out][6][n_veh] (may be NULL)
 * = MPC_delay_compensation_trajectory. */
int scpqp_delay_compensate(const scpqp_plant_params* p, int32_t B, double horizon, int32_t n_out,
                           const double* x_meas, const double* u_hold, const double* noise,
                           double* x0_out, double* traj_out, double h_max, void* stream);

/* Plant simulation of one MPC step (main.py:184-191): for every output tick
 * k = 0..n_ticks the reference restarts dopri5 at t0 from x_start and
 * integrates to t0 + k*tick with the constant control u_tick[b][v][k]
 * (= controlPathFullRes[v, ceil(t_k / tick) + 1]).  x_start [B][n_veh][6],
 * noise [B][n_veh][2] or NULL, x_path [B][n_veh][n_ticks+1][6]. */
int scpqp_plant_step(const scpqp_plant_params* p, int32_t B, int32_t n_ticks, double tick,
                     const double* x_start, const double* u_tick, const double* noise,
                     double* x_path, double h_max, void* stream);

/* Steering-limit enforcement (main.py:164-174), in place on the solver's
 * vehicle-major controls u[b*ld + v*hp + j]: U[0] clamped to +-umax and to
 * u0 +- du_lim, U[j] to +-umax and U[j-1] +- du_lim.  u0, umax: [B][n_veh]. */
int scpqp_clip_controls(int32_t B, int32_t n_veh, int32_t hp, int32_t ld, double du_lim, double* u,
                        const double* u0, const double* umax, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* SCPQP_H */
