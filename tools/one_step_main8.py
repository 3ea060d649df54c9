"""Diagnostic: the first closed-loop steps of main.py's own configuration (8 vehicles,
Hp 10) on a given build of the library (tests/closed_loop_check.py case main8).
    python tools/one_step_main8.py <lib.so> [steps]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"),
                os.path.join(ROOT, "senquential-convex-programming-for-trajectory-planning_amd")]


def main():
    import torch
    from scpqp import _lib
    _lib.use_build(sys.argv[1])
    import closed_loop_check as CC
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    dev = torch.device("cuda", 0)
    x_init, recs = CC.run_device("main8", 1, steps, dev)
    torch.cuda.synchronize()
    print("ok", sys.argv[1], steps, "steps")


if __name__ == "__main__":
    main()
