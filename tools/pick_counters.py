"""Pick one rocprofv3 PMC pass of matrix-core (MFMA) and VALU-activity counters from
the `rocprofv3 -L` listing of the box (counter names differ between ROCm releases).

    python tools/pick_counters.py counters_list.txt   ->  space-separated names (maybe empty)

At most 8 SQ counters (one pass, MI355X_MICROARCH.md rocprofv3 slots); the wave-cycle
counter rides along so the pass is self-normalising.
"""
import re
import sys

WANT = [
    "SQ_INSTS_VALU_MFMA_F64", "SQ_INSTS_VALU_MFMA_MOPS_F64", "SQ_VALU_MFMA_BUSY_CYCLES",
    "SQ_INSTS_MFMA", "SQ_ACTIVE_INST_MFMA", "SQ_INSTS_VALU_FMA_F64", "SQ_ACTIVE_INST_VALU",
    "SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES",
]


def main():
    try:
        text = open(sys.argv[1]).read()
    except OSError:
        print("")
        return
    have = set(re.findall(r"\b(SQ_[A-Z0-9_]+)\b", text))
    pick = [c for c in WANT if c in have][:8]
    print(" ".join(pick))


if __name__ == "__main__":
    main()
