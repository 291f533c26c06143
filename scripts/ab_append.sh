for r in 1 2; do ONLY=append KB_ARGS="--rounds 6" bash scripts/exp_run.sh || exit 1; done
