set -u
for r in 1 2; do for v in 0 1 2; do
out=$(MICLIP_ATTN=$v timeout -k 10 120 python scripts/bench_ops.py --ops attention --batch 256 --tokens 50 --width 768 --iters 50 2>/dev/null | tail -1) || { echo fail; exit 1; }
echo "r$r attn=$v $out"; done; done
