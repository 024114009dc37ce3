#!/bin/bash
# One parameterised GPU-box script (run from the repo root under gpurun; every
# GPU step under its own time limit, steps chained so a failure ends the call).
#
#   tools/gpu.sh tests <tag> [pytest selection / args...]   pytest -m gpu (+ smoke when no selection)
#   tools/gpu.sh smoke <tag>                                __graft_entry__.smoke()
#   tools/gpu.sh bench <tag> [bench args...]                one bench line -> <tag>/bench.json
#   tools/gpu.sh ab <tag> <rounds> "<libA> <libB>" [bench args...]
#                                                           exp_build variants alternated (tools/lib_ab.sh)
#   tools/gpu.sh prof <tag> [bench args...]                 rocprofv3 kernel trace + stats of a short bench
#   tools/gpu.sh pmc <tag> <kernels> [bench args...]        FETCH_SIZE / WRITE_SIZE passes -> pmc_config_d.json
#
# Several subcommands chain with "--":  tools/gpu.sh tests r04_a -- bench r04_a --steps 50
set -e
export PYTHONUNBUFFERED=1
run_one() {
  local cmd=$1 tag=$2; shift 2
  local out=gpurun_out/$tag
  mkdir -p $out
  case $cmd in
  tests)
    local -a sel=("$@")
    [ ${#sel[@]} -eq 0 ] && sel=(tests)
    timeout -k 10 1500 python -u -m pytest "${sel[@]}" -m gpu -x -v --timeout 600 --timeout-method thread \
        > $out/pytest_gpu.log 2>&1 || { tail -60 $out/pytest_gpu.log; return 1; }
    tail -3 $out/pytest_gpu.log
    if [ $# -eq 0 ]; then run_one smoke $tag; fi ;;
  smoke)
    timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 \
        || { tail -30 $out/smoke.log; return 1; }
    tail -3 $out/smoke.log ;;
  bench)
    timeout -k 10 900 python -u bench.py --detail-out $out/bench_detail.json "$@" > $out/bench.json 2> $out/bench.err \
        || { tail -30 $out/bench.err; return 1; }
    python3 tools/bench_brief.py $out/bench.json ;;
  ab)
    local rounds=$1 libs=$2; shift 2
    bash tools/lib_ab.sh $tag $rounds "$libs" "$@" ;;
  prof)
    (cd /tmp && export TMPDIR=/tmp)
    export TMPDIR=/tmp
    timeout -k 10 600 rocprofv3 --kernel-trace --stats -f csv -T -d $out/kt -o run -- python3 bench.py "$@" \
        > $out/kt_bench.json 2> $out/kt.err || { tail -30 $out/kt.err; return 1; }
    local kt=$(find $out/kt -name 'run_kernel_stats.csv' | head -1)
    head -25 $kt ;;
  pmc)
    export TMPDIR=/tmp
    local kernels=$1; shift
    for c in FETCH_SIZE WRITE_SIZE; do
      timeout -s KILL 180 rocprofv3 --pmc $c -f csv -T -d $out/pmc_$c -o run -- python3 bench.py "$@" \
          > $out/pmc_$c.json 2> $out/pmc_$c.err || { tail -20 $out/pmc_$c.err; return 1; }
    done
    local src=$(python3 -c "import sys; sys.path.insert(0, 'deneva-plus_amd'); from dvcc import _lib; print(_lib.source_hash())")
    python3 tools/pmc_summary.py $(find $out/pmc_FETCH_SIZE -name '*counter_collection.csv' | head -1) \
        $(find $out/pmc_WRITE_SIZE -name '*counter_collection.csv' | head -1) $out/pmc_config_d.json \
        $kernels config=D cc=NO_WAIT n_gpus=1 src_hash=$src > /dev/null
    echo "pmc summary: $out/pmc_config_d.json" ;;
  *)
    echo "unknown subcommand $cmd"; return 2 ;;
  esac
}
# split the arguments at "--" into subcommand invocations
args=()
for a in "$@"; do
  if [ "$a" == "--" ]; then run_one "${args[@]}"; args=(); else args+=("$a"); fi
done
[ ${#args[@]} -gt 0 ] && run_one "${args[@]}"
