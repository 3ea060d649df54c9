"""Build the per-config SQ counter record bench.py reads (profiles/rNN_pmc_sq_<cfg>.json)
from tools/gpu.sh pmc's pmc_sq_<cfg>.txt and pmc_mfma_<cfg>.txt (tools/pmc_table.py output).

    python tools/pmc_record.py <measure dir> <cfg> <kernel label> <session tag> > profiles/r03_pmc_sq_<cfg>.json
"""
import json
import os
import sys


def table(path):
    out, disp = {}, None
    for line in open(path):
        parts = line.split()
        if len(parts) >= 2 and parts[0].startswith("SQ_"):
            out[parts[0]] = float(parts[1])
            if "(" in line:
                disp = int(line.split("(")[1].split()[0])
    return out, disp


def main():
    d, cfg, label, tag = sys.argv[1:5]
    sq, disp = table(os.path.join(d, f"pmc_sq_{cfg}.txt"))
    mf, _ = table(os.path.join(d, f"pmc_mfma_{cfg}.txt"))
    mfma = mf.get("SQ_INSTS_VALU_MFMA_F64", 0.0)
    busy = mf.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0)
    rec = {
        "kernel": label,
        "dispatches": disp,
        "counters": sq,
        "lds_bank_conflict_ratio": sq["SQ_LDS_BANK_CONFLICT"] / sq["SQ_LDS_IDX_ACTIVE"],
        "wait_any_frac": sq["SQ_WAIT_ANY"] / sq["SQ_WAVE_CYCLES"],
        "valu_insts_per_wave": sq["SQ_INSTS_VALU"] / sq["SQ_WAVES"],
        "mfma_counters": mf,
        "mfma_f64_insts": mfma,
        # v_mfma_f64_16x16x4_f64: 16 x 16 x 4 multiply-adds = 2048 FLOP per wave instruction
        "mfma_f64_flops": 2048.0 * mfma,
        "mfma_busy_cycles_per_inst": busy / mfma if mfma else None,
        "note": (f"rocprofv3 --kernel-trace --pmc, one 8-counter SQ pass and one MFMA/VALU pass, "
                 f"bench.py --config {cfg} --steps 2 --warmup 1 --no-cpu; per-dispatch means "
                 f"(tools/pmc_table.py), shipped library (tools/gpu.sh pmc {tag})"),
    }
    json.dump(rec, sys.stdout, indent=1)


if __name__ == "__main__":
    main()
