set -u
for round in 1 2; do
  for s in c5 c4_1gpu_2e23; do
    echo "== round $round $s"
    timeout -k 10 200 python3 scripts/seq_probe.py --rings 2 --n 6 --shape $s --ab-lib $PWD/build_exp/libapus_seg3.so 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
