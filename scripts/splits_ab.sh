# Whole-step splits A/B (2 vs 3 vs 4 streams), 2 interleaved rounds -> gpurun_out/splits/
set -o pipefail
export MICLIP_QUIET=1
mkdir -p gpurun_out/splits
for r in 1 2; do for sp in 2 3 4; do
  out=$(timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-profile --splits $sp 2>/dev/null | tail -1) || { echo "bench failed ($sp)"; exit 1; }
  echo "splits $sp $(echo "$out" | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["value"], d["ms_per_step"], d["config"]["splits"], "clock", d.get("clock_ghz"))')" | tee -a gpurun_out/splits/ab.txt
done; done
