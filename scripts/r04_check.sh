#!/bin/bash
# r04 GPU check: named pytest groups, each under its own time limit; stops at
# the first crash / abort / timeout (pytest's 1 = "tests failed" continues).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/${OUT:-r04}
mkdir -p "$out"
run() {
  local name=$1 limit=$2; shift 2
  echo "=== $name: $*"
  timeout -k 10 "$limit" "$@" > "$out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -n 4 "$out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
PYT="python -u -m pytest -x -q -s -rf --timeout 300 --timeout-method thread"
for step in "$@"; do
  case $step in
    parity)  run parity 700 $PYT tests/test_gpu_parity.py tests/test_gpu_openclip.py ;;
    large)   run large 500 $PYT tests/test_gpu_largebatch.py tests/test_gpu_lnfold.py ;;
    drivers) run drivers 500 $PYT tests/test_gpu_drivers.py tests/test_gpu_distributed.py ;;
    kernels) run kernels 600 $PYT tests/test_gpu_kernels.py tests/test_gpu_mx.py ;;
    gpu)     run gpu 1100 $PYT -m gpu tests ;;
    gemm4s)  run gemm4s 600 $PYT tests/test_gpu_gemm4s.py ;;
    ops4s)   run ops4s 400 python scripts/bench_ops.py --ops gemm --variants 259,508,516,259,508,516 --iters 20 ;;
    diag4s)  run diag4s 400 python scripts/bench_ops.py --ops gemm --only fc,proj --variants 508,508d,508e,259,259d,508,508d,508e,259 --iters 20 ;;
    spread)  run spread 400 python scripts/bench_ops.py --ops gemm --only fc,proj --variants 259,508,530,531,532,533,534,259,508,530,531,532,533,534 --iters 20 ;;
    abgemm)  run abgemm 500 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-profile --ab-gemm 0:0,508:0,516:0,508:508 ;;
    lnfix)   run lnfix 600 $PYT tests/test_gpu_lnfold.py tests/test_gpu_openclip.py tests/test_gpu_parity.py -k "benched or head or zero_shot" ;;
    smoke)   run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench)   run bench 400 python bench.py --steps 10 --warmup 3 --cpu-seconds 5 ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
