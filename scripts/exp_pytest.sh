#!/bin/bash
# the GPU parity tests against an experiment build: bash scripts/exp_pytest.sh NAME [pytest args]
set -u
cd "$(dirname "$0")/.."
name=$1; shift
APUS_GPU_LIB=$PWD/build_exp/libapus_$name.so timeout -k 10 600 python3 -u -m pytest "$@" -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread
