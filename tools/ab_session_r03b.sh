set -e
echo "== C2 cold: base (CAS after answers), store-first CAS, store-first no-return CAS, plain-store raises"
ROUNDS=2 ARGS="--config c2 --secondary none" LIBS="tools/ab/libsketch_base.so tools/ab/libsketch_storefirst.so tools/ab/libsketch_k1nr.so tools/ab/libsketch_k1st.so" bash tools/ab_passes.sh
echo "== C3: default (small counter table) vs pa_grid=2 (2048-entry table)"
ROUNDS=3 OPTS=" ;--opt pa_grid=2" bash tools/ab_opts.sh
