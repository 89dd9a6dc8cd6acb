# Bench lines for C2 / C4 / C5 on the final tree (parity already green) -> gpurun_out/configs/
set -o pipefail
export MICLIP_QUIET=1
mkdir -p gpurun_out/configs
timeout -k 10 300 python bench.py --model ViT-B/32 --dtype bf16 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/configs/c2.json 2> gpurun_out/configs/c2.err || exit 1
timeout -k 10 300 python bench.py --model ViT-L/14@336px --dtype fp16 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/configs/c4.json 2> gpurun_out/configs/c4.err || exit 1
timeout -k 10 300 python bench.py --model ViT-H-14 --dtype mxfp8 --batch 512 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/configs/c5.json 2> gpurun_out/configs/c5.err || exit 1
for c in c2 c4 c5; do python3 -c "import json; d=json.loads(open('gpurun_out/configs/$c.json').read().strip().splitlines()[-1]); print('$c', d['value'], d['ms_per_step'], d['path_mfma_frac'], d['roofline'].get('clock_ghz'))"; done
