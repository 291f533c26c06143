#!/bin/bash
# the scalar kernel's phases from the APUS_EXP_QTIME build (scripts/scalar_phases.py)
set -u
cd "$(dirname "$0")/.."
APUS_GPU_LIB=$PWD/build_exp/libapus_qtime.so timeout -k 10 120 python3 scripts/scalar_phases.py
