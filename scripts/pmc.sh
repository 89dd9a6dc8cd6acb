#!/bin/bash
# PMC counter passes (one rocprofv3 run per counter group, kernel-trace only, no
# other tracing). Output: gpurun_out/pmc/<pass>/
#   pmc.sh            -> occupancy / MFMA / LDS / L2 groups over the fc+proj GEMMs
#   pmc.sh traffic    -> FETCH_SIZE and WRITE_SIZE over gemm_fc, then scripts/traffic.py
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
pass() {
  local name=$1; shift
  local ctrs=$1; shift
  echo "=== pass $name: $ctrs"
  timeout -k 10 300 rocprofv3 --pmc $ctrs --kernel-trace --output-format csv \
      -d "$PWD/gpurun_out/pmc/$name" -o run -- "$@" > "gpurun_out/pmc/$name.log" 2>&1
  local rc=$?
  echo "pass $name rc=$rc"; tail -3 "gpurun_out/pmc/$name.log"
  if [ $rc -ne 0 ]; then echo "stopping"; exit $rc; fi
}
if [ "${1:-}" = traffic ]; then
  CMD=(python3 bench.py --steps 2 --warmup 1 --splits 1 --no-cpu-baseline --no-profile)
  pass fetch FETCH_SIZE "${CMD[@]}"
  pass write WRITE_SIZE "${CMD[@]}"
  python3 scripts/traffic.py
  exit $?
fi
if [ "${1:-}" = attn ]; then
  CMD=(python3 scripts/bench_ops.py --ops attention --iters 5)
  i=0
  for grp in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE" \
             "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU" \
             "SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_SCA SQ_INSTS_VALU_TRANS_F32"; do
    i=$((i+1))
    pass "b$i" "$grp" "${CMD[@]}"
  done
  exit 0
fi
if [ "${1:-}" = bench ]; then
  # every kernel of the benched step (one unsplit step: --splits 1)
  # PMC_BENCH_ARGS: extra bench.py arguments (e.g. "--model ViT-L/14@336px" for C4)
  CMD=(python3 bench.py --steps 1 --warmup 0 --splits 1 --no-cpu-baseline --no-profile ${PMC_BENCH_ARGS:-})
  i=0
  for grp in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE" \
             "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_SALU" \
             "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM" ; do
    i=$((i+1))
    pass "b$i" "$grp" "${CMD[@]}"
  done
  exit 0
fi
CMD=(python3 scripts/bench_ops.py --ops gemm --only fc,proj --variants 0 --iters 5)
i=0
for grp in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE" \
           "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F16 SQ_INSTS_LDS SQ_WAIT_INST_LDS" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_UNALIGNED_STALL" \
           "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  pass "p$i" "$grp" "${CMD[@]}"
done
