#!/usr/bin/env python
"""HBM-side bytes per launch of the MLP c_fc GEMM from two rocprofv3 PMC passes.

Reads gpurun_out/pmc/{fetch,write}/run_counter_collection.csv written by
`scripts/pmc.sh traffic` (bench.py itself with --splits 1, so every c_fc launch
is the M=65792 N=4096 K=1024 launch the bench's profiled step times) and writes
profiles/traffic_gemm_fc.json, which bench.py reports as roofline.traffic only
when model, dtype, epilogue and M match the run.

Corrections (MI355X_MICROARCH.md, HBM section): FETCH_SIZE and WRITE_SIZE are
KiB; on gfx950 FETCH_SIZE tallies 128-B streaming reads at 64 B, so it is
doubled; WRITE_SIZE is exact for 16-B/lane stores. Both count L2 memory-side
requests, i.e. Infinity-Cache hits are included (an upper bound on HBM bytes).
"""
import csv
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
M, N, K = 65792, 4096, 1024


EPI = os.environ.get("MICLIP_TRAFFIC_EPI", "EpiStoreLN")   # the c_fc epilogue profiled


def launches(path, counter):
    """Per-dispatch values of `counter` for the QuickGELU-epilogue 256x256
    GEMM launches (<EPI><T, 1>: the c_fc GEMM) of the largest grid in the file
    (the persistent grid of M = 65792)."""
    rows = []
    tag = f"{len(EPI)}{EPI}IDF16_Li1E"
    with open(path) as f:
        for r in csv.DictReader(f):
            if (r["Counter_Name"] == counter and ("gemm256_kernel" in r["Kernel_Name"] or "gemm256s_kernel" in r["Kernel_Name"])
                    and tag in r["Kernel_Name"]):
                rows.append((int(r["Grid_Size"]), float(r["Counter_Value"])))
    if not rows:
        return []
    g = max(x[0] for x in rows)
    return [v for gs, v in rows if gs == g]


def main():
    d = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "gpurun_out", "pmc")
    fetch = launches(os.path.join(d, "fetch", "run_counter_collection.csv"), "FETCH_SIZE")
    write = launches(os.path.join(d, "write", "run_counter_collection.csv"), "WRITE_SIZE")
    if not fetch or not write:
        sys.exit("no gemm_fc launches found in the PMC passes")
    rd = 2.0 * 1024 * statistics.median(fetch)
    wr = 1024 * statistics.median(write)
    algo = 2 * M * K + 2 * N * K + 2 * M * N
    out = {"kernel": "gemm_fc", "epilogue": EPI, "model": "ViT-L/14", "dtype": "fp16",
           "batch": 256, "M": M, "N": N, "K": K,
           "source": os.environ.get("MICLIP_TRAFFIC_SOURCE", "profiles/r02/pmc_traffic"),
           "hbm_bytes_per_launch": round(rd + wr), "read_bytes": round(rd), "write_bytes": round(wr),
           "algorithmic_bytes": algo, "launches": [len(fetch), len(write)],
           "method": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes), KiB x1024, "
                     "FETCH_SIZE x2 (gfx950 128-B requests tallied at 64 B); median over launches"}
    with open(os.path.join(ROOT, "profiles", "traffic_gemm_fc.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
