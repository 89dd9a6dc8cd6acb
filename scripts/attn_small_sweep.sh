# Attention variants at C2's shape (ViT-B/32 bs=256: N = 50, 12 heads of 64) and the CLS
# block pieces, op level -> gpurun_out/attn_small/
set -o pipefail
export MICLIP_QUIET=1
mkdir -p gpurun_out/attn_small
timeout -k 10 200 python scripts/bench_ops.py --ops attention --batch 256 --tokens 50 --width 768 --attn-variants 0,1,2,4,10,12,16,0,1,2 > gpurun_out/attn_small/ops.jsonl || exit 1
cat gpurun_out/attn_small/ops.jsonl
