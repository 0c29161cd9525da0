#!/bin/bash
set -u
O=gpurun_out/r02h
mkdir -p $O
export TMPDIR=/tmp
scripts/guard.sh 400 $O/pytest_host.log python -u -m pytest tests/test_host.py -m gpu -v --timeout 200 --timeout-method thread || exit $?
