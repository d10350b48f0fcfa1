#!/bin/bash
# GPU session: the -m gpu suite, then the default bench (each step time-bounded; stop on a crash).
#   tools/gpu_session.sh [tag] [pytest selection...]   (KSEL: a pytest -k expression; NO_BENCH=1: tests only)
set -o pipefail
tag=${1:-s}; shift
sel=${@:-tests}
mkdir -p gpurun_out
export MMPFN_PARITY_LOG=$PWD/gpurun_out/parity_$tag.jsonl
kargs=(); [ -n "$KSEL" ] && kargs=(-k "$KSEL")
timeout -k 10 900 python -u -m pytest $sel "${kargs[@]}" -m gpu -v -s --timeout 300 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/pytest_$tag.log 2>&1
rc=$?
echo "pytest_rc=$rc" >> gpurun_out/pytest_$tag.log
grep -E "passed|failed|error" gpurun_out/pytest_$tag.log | tail -3
case $rc in 0|1) ;; *) exit $rc ;; esac
[ -n "$NO_BENCH" ] && exit $rc
timeout -k 10 600 python -u bench.py $BENCH_ARGS > gpurun_out/bench_$tag.json 2> gpurun_out/bench_$tag.err || exit 1
cat gpurun_out/bench_$tag.json
exit $rc
