# ablation timing of the fp6 GEMMs (development; build/f6b_abl<N> built with -DF6_ABL=N)
for b in "$@"; do
  echo "== $b"; timeout -k 10 60 ./$b 20 | grep -E "TOPS" || exit 1
done
