#!/bin/bash
# r04: fp16 residual stream under bf16 compute -- parity (bf16 configs), large-batch C2,
# drivers, then C2 same-process A/B against the fp32 stream (options resid_f32)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/${OUT:-r04bf}
mkdir -p "$out"
export MICLIP_QUIET=1
PYT="python -u -m pytest -x -q -s -rf --timeout 300 --timeout-method thread"
step() { local n=$1 t=$2; shift 2; echo "=== $n"; timeout -k 10 "$t" "$@" > "$out/$n.log" 2>&1; local rc=$?; echo "$n rc=$rc"; tail -n 3 "$out/$n.log"; [ $rc -eq 0 ] || exit $rc; }
step parity 600 $PYT tests/test_gpu_parity.py tests/test_gpu_largebatch.py -k "bf16 or fp32_residual or vitb32"
step ab 400 python bench.py --model ViT-B/32 --dtype bf16 --steps 10 --warmup 3 --no-cpu-baseline --ab-options resid_f32=1
step graph 300 python scripts/graph_probe.py 256 ViT-B/32 bf16
