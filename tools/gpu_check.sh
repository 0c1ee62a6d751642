#!/bin/bash
# GPU check used during development: parity tests then a short bench.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests -m gpu -x -q > gpurun_out/tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline "$@" > gpurun_out/bench.log 2>&1
