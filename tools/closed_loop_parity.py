"""Closed-loop parity record (profiles/r02_closed_loop_<case>.json): the device
ClosedLoopBatch against the CPU restatement over the reference's Nsim = 50
steps (tests/closed_loop_check.py does the work).

    python tools/closed_loop_parity.py main8 1 50      # main.py:234-255 configuration
    python tools/closed_loop_parity.py c2 16 50        # 16 perturbed c2 realisations
    (main8, or --rk4: also the restated loop on the device's RK4 integrator)
"""
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path[:0] = [os.path.join(ROOT, "tests"), ROOT]

import closed_loop_check as CC  # noqa: E402


def main():
    case = sys.argv[1] if len(sys.argv) > 1 else "main8"
    B = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    steps = int(sys.argv[3]) if len(sys.argv) > 3 else 50
    out = sys.argv[4] if len(sys.argv) > 4 else f"gpurun_out/closed_loop_{case}.json"
    t = time.time()
    mirror = range(steps) if case == "main8" else ()
    # main8: also the restated loop on the device's RK4 integrator (closed_loop_check 3.)
    per = CC.run(case, B, steps, "cuda", workers=16, mirror_steps=mirror,
                 rk4_loop=case == "main8" or "--rk4" in sys.argv)
    s = CC.summary(per)
    s.update(case=case, wall_s=time.time() - t)
    print(json.dumps(s, indent=1))
    os.makedirs(os.path.dirname(out) or ".", exist_ok=True)
    with open(out, "w") as f:
        json.dump(dict(summary=s, per_step=per), f, indent=1)


if __name__ == "__main__":
    main()
