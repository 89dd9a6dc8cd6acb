#!/bin/bash
# GPU-box check sequence: each step has its own time limit; a crash, abort or
# timeout (any status other than 0 or pytest's 1 = "tests failed") stops the run.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
run() {
  local name=$1 limit=$2; shift 2
  echo "=== $name: $*"
  timeout -k 10 "$limit" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -n 25 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
steps=("$@")
[ ${#steps[@]} -eq 0 ] && steps=(kernels parity bench)
for step in "${steps[@]}"; do
  case $step in
    kernels) run kernels 400 python -m pytest tests/test_gpu_kernels.py -q -rf ;;
    parity)  run parity 900 python -m pytest tests/test_gpu_parity.py -q -s -rf ;;
    gpu)     run gputests 1000 python -m pytest tests -m gpu -q -rf ;;
    smoke)   run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench)   run bench 600 python bench.py --steps 10 --warmup 3 ;;
    ops)     run ops 300 python scripts/bench_ops.py --variants 258 ;;
    outl)    run outl 300 python -m pytest tests/test_outliers.py -q -rf ;;
    pre)     run pre 300 python -m pytest tests/test_preprocess.py -q -rf ;;
    benchpre) run benchpre 300 python scripts/bench_preprocess.py ;;
    regepi)  run regepi 300 python scripts/bench_ops.py --ops gemm --variants 0,260,3,0,260,3 ;;
    blas)    run blas 300 python scripts/bench_ops.py --ops gemm --variants 0 --torch ;;
    attn)    run attn 200 python scripts/bench_ops.py --ops attention ;;
    group)   run group 300 python scripts/bench_ops.py --ops gemm --variants 1258,4258,8258,2258,1258,4258 ;;
    traffic) run traffic 700 bash scripts/pmc.sh traffic ;;
    ksweep)  run ksweep 300 python scripts/bench_ops.py --variants 0 --ksweep --ops gemm ;;
    prof)    export TMPDIR=/tmp
             run prof 600 rocprofv3 --kernel-trace --stats --output-format csv \
                 -d "$PWD/gpurun_out/prof" -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --splits 1 ;;
    benchq)  run benchq 400 python bench.py --steps 5 --warmup 2 --cpu-seconds 5 ;;
    benchab) run benchab 500 python bench.py --steps 8 --warmup 2 --no-cpu-baseline --ab-splits ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
