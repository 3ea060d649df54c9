"""Drop-in for the reference's ``Config.py`` (Config.py:1-26): solver settings.

Only ``Config().QCQP.constraintTolerance`` is read on the SCP path
(SCP_controller.py:194,244,260; Config.py:18).  ``MIP_CPLEX`` belongs to the
MIQP controller (out of scope) and is kept for import compatibility.
"""


class MIP_CPLEX:
    """MIQP settings (Config.py:4-10); unused by the SCP path."""

    def __init__(self):
        self.bigM = 1000
        self.R_Gain = 0.1
        self.polygonalNormApproximationDegree = 6
        self.timelimit = 300
        self.obstAsQCQP = 1


class QCQP:
    """QCQP settings (Config.py:12-18)."""

    def __init__(self):
        self.default_dsafeExtra = 0
        # constraint tolerance = 2 * d_safe * distance tolerance (~1 mm)
        self.constraintTolerance = 2 * 2.1 * 1e-3


class Config:
    def __init__(self):
        self.MIP_CPLEX = MIP_CPLEX()
        self.QCQP = QCQP()
        self.Lagrange_Mosek_R_Gain = 10
