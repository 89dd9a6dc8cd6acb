# Attention variants at C4's shape (ViT-L/14@336 bs=256: N = 577, 16 heads of 64), op level
set -o pipefail
export MICLIP_QUIET=1
mkdir -p gpurun_out/attn577
timeout -k 10 300 python scripts/bench_ops.py --ops attention --batch 256 --tokens 577 --width 1024 --attn-variants 0,1,10,11,12,13,14,15,16,0,1,12,16 > gpurun_out/attn577/ops.jsonl || exit 1
cat gpurun_out/attn577/ops.jsonl
