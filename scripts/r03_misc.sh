#!/bin/bash
# MX-fp8 epilogue probe, AsyncHostSink overlap, and the secondary BASELINE config lines.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export MICLIP_QUIET=1
O=gpurun_out/r03x
mkdir -p $O
timeout -k 10 120 python scripts/bench_ops.py --batch 128 --ops attention --attn-variants 8,10,8,10,8,10 > $O/attn_hm.jsonl 2>&1 && cat $O/attn_hm.jsonl \
  && timeout -k 10 200 python scripts/probe/mx_epi.py > $O/mx_epi.jsonl 2>&1 && cat $O/mx_epi.jsonl \
  && timeout -k 10 300 python scripts/bench_sink.py > $O/sink.json 2> $O/sink.err && cat $O/sink.json \
  && timeout -k 10 300 python bench.py --model ViT-B/32 --dtype bf16 --steps 10 --warmup 3 --no-cpu-baseline > $O/c2.json 2> $O/c2.err \
  && timeout -k 10 300 python bench.py --model ViT-L/14@336px --dtype fp16 --steps 5 --warmup 2 --no-cpu-baseline > $O/c4.json 2> $O/c4.err \
  && timeout -k 10 300 python bench.py --model ViT-H-14 --dtype mxfp8 --batch 512 --steps 5 --warmup 2 --no-cpu-baseline > $O/c5.json 2> $O/c5.err \
  && for c in c2 c4 c5; do python3 -c "import json,sys; d=json.loads(open('$O/$c.json').read().strip().splitlines()[-1]); print('$c', d['value'], d['ms_per_step'], d['path_mfma_frac'], d.get('clock_ghz'))"; done
