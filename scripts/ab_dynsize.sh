set -u
for r in 1 2; do
  for g in 2097152 4194304; do
    ONLY=wave_walk_checksum KB_ARGS="--groups $g --rounds 6" bash scripts/exp_run.sh || exit 1
  done
done
