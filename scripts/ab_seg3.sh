#!/bin/bash
# the segment walk against build_exp/libapus_prev.so (the build before it), the
# same rings in one process (seq_probe.py --ab-lib): C5 and the C4 1-GPU shape
set -u
cd "$(dirname "$0")/.."
for s in c5 c4_1gpu_2e23; do
  echo "== $s"
  python3 scripts/seq_probe.py --rings 2 --n 6 --shape $s --ab-lib $PWD/build_exp/libapus_prev.so 2>&1 | grep -v amdgpu.ids || exit 1
done
