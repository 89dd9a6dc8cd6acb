#!/bin/bash
# Stamps of the four GEMM shapes with the main-loop vmcnt waits split out
# (libstamp_gemm_kloop.so: segment "epi_barrier" = K-loop vmcnt wait there).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03s
mkdir -p $O
for s in fc qkv out proj; do
  STAMP_LIB=build/stamps/libstamp_gemm_kloop.so timeout -k 10 120 python scripts/stamps/run.py gemm --shape $s > $O/kloop_$s.json || exit 1
  timeout -k 10 120 python scripts/stamps/run.py gemm --shape $s > $O/plain_$s.json || exit 1
done
python3 - <<'PY'
import json
for s in ["fc","qkv","out","proj"]:
    for k in ["plain","kloop"]:
        d=json.load(open(f"gpurun_out/r03s/{k}_{s}.json"))
        print(s, k, d["ms"], d["clock_ghz_mean"], {n: v["share"] for n, v in d["segments"].items()})
PY
