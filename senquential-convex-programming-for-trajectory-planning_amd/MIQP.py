"""Import-compatibility stub for the reference's ``MIQP.py`` (MIQP.py:1-498).

main.py imports ``MIQPcontroller`` unconditionally (main.py:14) but only uses
it when ``controllerName == 'MIQP'``.  The mixed-integer controller needs a
MIP solver (CPLEX) and is outside the accelerated path (out of
scope); constructing it raises.
"""


class MIQPcontroller:
    def __init__(self, scenario, Iter, prevOutput):
        raise NotImplementedError(
            "MIQPcontroller is not part of the MI355X SCP-QP path; use SCPcontroller")
