# rocprofv3 kernel trace of the C2 (ViT-B/32 bf16 bs=256) bench -> gpurun_out/c2prof
set -o pipefail
export MICLIP_QUIET=1 TMPDIR=/tmp
mkdir -p gpurun_out/c2prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/c2prof/raw -o c2 --output-format csv -- python bench.py --model ViT-B/32 --dtype bf16 --steps 5 --warmup 2 --no-cpu-baseline --no-profile > gpurun_out/c2prof/bench.json 2> gpurun_out/c2prof/err.txt || exit 1
f=$(find gpurun_out/c2prof/raw -name '*kernel_stats.csv' | head -1); cp "$f" gpurun_out/c2prof/kernel_stats.csv
f=$(find gpurun_out/c2prof/raw -name '*kernel_trace.csv' | head -1); cp "$f" gpurun_out/c2prof/kernel_trace.csv
rm -rf gpurun_out/c2prof/raw
echo ok
