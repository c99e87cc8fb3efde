# Round 2, pass j: cost attribution on C2/C3/C4 by (inexact, measurement-only)
# variants: X1 sphere-root sqrt without scaling, X2 Philox 7 rounds, X3 ONB
# without normalisation, X4 Philox 5 rounds.
set -e
O=gpurun_out/r02j
mkdir -p $O
bash profiles/ab_variants.sh base X1 X2 X3 X4 base 2>&1 | tee $O/ab.log
