#!/usr/bin/env python
"""Per-kernel-class summary of the `scripts/pmc.sh bench` passes (gpurun_out/pmc/b*).

Sums every counter over the dispatches of each kernel symbol (the last
occurrence of each kernel in the single profiled step) and prints derived
ratios: MFMA busy per SIMD-cycle, wait / active fractions of wave cycles,
VALU:MFMA instruction ratio, LDS-array activity.
"""
import collections
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def short(name):
    for k in ("gemm256s_kernel", "attention_pipe_kernel", "attention_x8_kernel", "attention_kernel", "ln_stats_kernel",
              "layernorm_h2_kernel", "layernorm_kernel", "gemm_tail", "gemm256_kernel", "im2col",
              "zero_shot", "rows_matmul", "class_token", "gemm_nt_kernel"):
        if k in name:
            for epi in ("EpiStoreLN", "EpiResidual", "EpiStore", "EpiPatch", "EpiF32"):
                if epi in name:
                    act = "1" if "Li1E" in name else ("2" if "Li2E" in name else "0")
                    return f"{k}<{epi}{',' + act if 'Store' in epi else ''}>"
            return k
    return name[:60]


def main():
    d = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "gpurun_out", "pmc")
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for path in sorted(glob.glob(os.path.join(d, "b*", "run_counter_collection.csv"))):
        with open(path) as f:
            for r in csv.DictReader(f):
                k = short(r["Kernel_Name"])
                acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
                disp[k].add((os.path.basename(os.path.dirname(path)), r["Dispatch_Id"]))
    out = {}
    for k, c in sorted(acc.items(), key=lambda kv: -kv[1].get("GRBM_GUI_ACTIVE", 0)):
        g = c.get("GRBM_GUI_ACTIVE", 0)
        wc = c.get("SQ_WAVE_CYCLES", 0)
        row = {"dispatches_per_pass": len(disp[k]) // 3 or len(disp[k]),
               "gui_active_cycles": g,
               # SQ_VALU_MFMA_BUSY_CYCLES is summed over the chip's SIMDs (1024); GRBM over 8 XCDs
               "mfma_busy_per_simd": (c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / 1024) / (g / 8) if g else None,
               "wait_any_frac": c.get("SQ_WAIT_ANY", 0) / wc if wc else None,
               "wait_inst_any_frac": c.get("SQ_WAIT_INST_ANY", 0) / wc if wc else None,
               "active_inst_frac": c.get("SQ_ACTIVE_INST_ANY", 0) / wc if wc else None,
               "valu_per_mfma": c.get("SQ_INSTS_VALU", 0) / c["SQ_INSTS_MFMA"] if c.get("SQ_INSTS_MFMA") else None,
               "lds_per_mfma": c.get("SQ_INSTS_LDS", 0) / c["SQ_INSTS_MFMA"] if c.get("SQ_INSTS_MFMA") else None,
               "lds_idx_active_per_cu": (c.get("SQ_LDS_IDX_ACTIVE", 0) / 256) / (g / 8) if g else None,
               "lds_bank_conflict": c.get("SQ_LDS_BANK_CONFLICT", 0),
               "wait_inst_lds_frac": c.get("SQ_WAIT_INST_LDS", 0) / wc if wc else None,
               "active_valu_frac": c.get("SQ_ACTIVE_INST_VALU", 0) / wc if wc else None,
               "active_lds_frac": c.get("SQ_ACTIVE_INST_LDS", 0) / wc if wc else None,
               "active_sca_frac": c.get("SQ_ACTIVE_INST_SCA", 0) / wc if wc else None,
               "trans_per_mfma": c.get("SQ_INSTS_VALU_TRANS_F32", 0) / c["SQ_INSTS_MFMA"] if c.get("SQ_INSTS_MFMA") else None,
               "waves_per_simd_avg": c.get("SQ_WAVE_CYCLES", 0) / (g / 8 * 1024) if g else None}
        out[k] = {a: (round(b, 4) if isinstance(b, float) else b) for a, b in row.items()}
        print(k, json.dumps(out[k]))
    return out


if __name__ == "__main__":
    main()
