"""Algorithmic FP64 FLOP count of the executed algorithm (roofline numerator).

SURVEY.md §8(d) prices the dense-KKT Mehrotra IPM as
``F_ipm(n, m) = m n^2 + n^3/3 + 8 m n + 4 n^2``.  The HIP kernel does not run
that algorithm: it assembles the normal matrix from the Toeplitz structure
(``K_uu = B'(2Q + W)B + diag``) and factors it as L D L'.  As
§8(d) requires, the count below restates F for the executed algorithm.  An FMA
counts as 2 FLOPs.  Only arithmetic the algorithm needs is counted (no
padding, no redundant lanes); the numbers are per problem and use the
per-problem SCP / IPM iteration counts the kernel returns.

Symbols: V vehicles, H horizon, O obstacles, N = V H controls, n = N + 1
QP variables (slack omega last), m = (V(V-1)/2 + V O) H constraint rows,
mc = m + 2N + 1 inequality rows (collision rows, two box rows per control,
omega >= 0).
"""
from __future__ import annotations


def _sizes(V, H, O):
    N = V * H
    n = N + 1
    m = (V * (V - 1) // 2 + V * O) * H
    mc = m + 2 * N + 1
    return N, n, m, mc


def toeplitz_apply(V, H):
    """calB x or calB' y: per vehicle a lower-triangular Toeplitz product with 2-vector blocks."""
    return 2 * 2 * V * H * (H + 1) // 2


def assemble(V, H, O):
    """K = P + G' D G from the W~ blocks (12 FLOPs per (k, l, l') term of a 2x2 quadratic form)."""
    N, n, m, mc = _sizes(V, H, O)
    s_off = sum((H - mm) * (2 * mm + 1) for mm in range(H))   # sum_{l,l'} (H - max(l,l'))
    s_diag = sum((H - l) * (l + 1) for l in range(H))          # sum_{l>=l'} (H - l)
    pairs = V * (V - 1) // 2
    kuu = 12 * (pairs * s_off + V * s_diag)
    wblocks = 6 * H * (V * (V - 1 + O) + pairs)
    omega = toeplitz_apply(V, H) + 4 * V * H * (V - 1 + O) + 3 * m
    return kuu + wblocks + omega + 4 * N


def factor(n):
    """L D L' of the n x n normal matrix."""
    return n ** 3 // 3


def solve(n):
    """Forward + diagonal + backward substitution."""
    return 2 * n * n + n


def g_apply(V, H, O):
    N, n, m, mc = _sizes(V, H, O)
    return toeplitz_apply(V, H) + 6 * m + 2 * N


def gt_apply(V, H, O):
    N, n, m, mc = _sizes(V, H, O)
    return 4 * V * H * (V - 1 + O) + 2 * m + toeplitz_apply(V, H) + 2 * N


def ipm_iteration(V, H, O):
    N, n, m, mc = _sizes(V, H, O)
    residuals = 2 * toeplitz_apply(V, H) + 4 * V * H * (V - 1 + O) + 8 * m + 12 * mc + 8 * N
    newton = gt_apply(V, H, O) + solve(n) + g_apply(V, H, O) + 12 * mc
    return residuals + mc + assemble(V, H, O) + factor(n) + 2 * newton + 20 * mc


def qp_init(V, H, O):
    """CVXOPT initial point of a cold QP: assemble + factor + one solve + G x."""
    N, n, m, mc = _sizes(V, H, O)
    return assemble(V, H, O) + factor(n) + gt_apply(V, H, O) + solve(n) + g_apply(V, H, O) + 8 * mc


def polish_round(V, H, O):
    """One active-set polish round: assemble + factor + certification / correction."""
    N, n, m, mc = _sizes(V, H, O)
    return assemble(V, H, O) + factor(n) + 6 * mc


def polish_refine(V, H, O):
    """One multiplier-iteration step: G' t, solve, G x - h, dual update, step norm."""
    N, n, m, mc = _sizes(V, H, O)
    return gt_apply(V, H, O) + solve(n) + g_apply(V, H, O) + 6 * mc + 2 * n


def scp_iteration_extra(V, H, O):
    """Constraint linearisation + QCQP evaluation (once per SCP iteration)."""
    N, n, m, mc = _sizes(V, H, O)
    rows = toeplitz_apply(V, H) + m * (20 + 2 * 4 * (H + 1) // 2 * 2)
    evaluate = toeplitz_apply(V, H) + 8 * m + 8 * N
    return rows + evaluate


def setup(V, H):
    """Jacobian + 8x8 Pade-13 expm (6 products + 8x8 solve + 1 squaring) + recursions + Psi0."""
    expm = 7 * 2 * 8 ** 3 + 2 * 8 ** 3 * 2
    return V * (expm + 2 * H * 72 + 2 * H * (H + 1) + 200)


def problem_flops(V, H, O, n_scp, n_ipm, n_polish, n_refine, n_warm):
    """FP64 FLOPs of one SCP solve from the counters the kernel returns: QPs (n_scp),
    IPM iterations, polish rounds, multiplier-iteration solves and warm-certified QPs
    (which skip the IPM initial point)."""
    cold = n_scp - n_warm
    return (setup(V, H) + toeplitz_apply(V, H) + n_scp * scp_iteration_extra(V, H, O)
            + cold * qp_init(V, H, O) + n_ipm * ipm_iteration(V, H, O)
            + n_polish * polish_round(V, H, O) + n_refine * polish_refine(V, H, O))


def batch_flops(V, hps, O, n_scp, n_ipm, n_polish, n_refine, n_warm):
    """Sum over a batch (arrays of per-problem horizon / counters)."""
    tot = 0
    for H, s, i, p, r, w in zip(hps, n_scp, n_ipm, n_polish, n_refine, n_warm):
        tot += problem_flops(V, int(H), O, int(s), int(i), int(p), int(r), int(w))
    return tot


def dense_ipm_reference(n, m):
    """SURVEY.md §8(d) dense-KKT IPM iteration count, for comparison in DESIGN.md."""
    return m * n * n + n ** 3 // 3 + 8 * m * n + 4 * n * n


def survey_dense_problem(V, H, O, n_scp, n_ipm):
    """SURVEY.md §8(d)'s solver-independent count of one SCP solve at the measured
    counts: F_setup + sum_s [F_row + F_eval + k_ipm,s F_ipm(n, m)], with
    F_ipm(n, m) = m n^2 + n^3/3 + 8 m n + 4 n^2 over the m linearised rows (the
    formula's m), F_row = 2 V H^2 + m (4H + 8), F_eval = 2 V H^2 + 6 m and
    F_setup = V (2 F_expm7 + 144 H + 4 H^3), F_expm7 = 14 * 2 * 7^3.  It does not
    depend on how the kernel solves the QP, so more polish work cannot raise it."""
    N = V * H
    n = N + 1
    m = (V * (V - 1) // 2 + V * O) * H
    f_row = 2 * V * H * H + m * (4 * H + 8)
    f_eval = 2 * V * H * H + 6 * m
    f_setup = V * (2 * 14 * 2 * 7 ** 3 + 144 * H + 4 * H ** 3)
    return f_setup + n_scp * (f_row + f_eval) + n_ipm * dense_ipm_reference(n, m)


def survey_dense_batch(V, hps, O, n_scp, n_ipm):
    return sum(survey_dense_problem(V, int(H), O, int(s), int(i))
               for H, s, i in zip(hps, n_scp, n_ipm))


def compulsory_bytes(V, H, O):
    """HBM bytes a problem must move: inputs x0, u0, noise (+ obstacles) and outputs u, traj, scalars."""
    N = V * H
    inp = 8 * (6 * V + V + 2 * V + 2 * O * H)
    out = 8 * (N + 2 * H * V) + 3 * 8 + 4 * 4
    return inp + out
