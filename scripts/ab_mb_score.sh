cd /root/repo
for i in 1 2; do for v in ${VARIANTS:-cur skip_epi}; do for L in 0 16000 6400; do
  EWK_FIXED_LEN=$L EWK_LIB=$PWD/variants/$v.so timeout -k 10 120 python3 scripts/mb_score.py 65536 10 2>&1 | grep Gframes || exit 1
done; done; done
