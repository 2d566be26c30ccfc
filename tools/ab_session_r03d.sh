set -e
echo "== C2 (descriptors prebuilt)"
ROUNDS=3 ARGS="--config c2" OPTS=" " bash tools/ab_opts.sh
