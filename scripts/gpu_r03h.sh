#!/bin/bash
# Experiment: is the small-|mean| score error the float32 DCT?  variants/*.so (b: fp64 DCT)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for f in variants/*.so; do
  echo "== $(basename $f)"
  EWK_LIB=$PWD/$f timeout -k 10 300 python scripts/fuzz_case_stats.py 33:187:1000 31:113:1000 31:113:1 2>&1 | grep seed
  EWK_LIB=$PWD/$f timeout -k 10 300 python scripts/fuzz_err.py 33 200 1000 2>&1 | grep -E "fuzz|DIFFERS"
  EWK_LIB=$PWD/$f timeout -k 10 400 python scripts/std_norm_dist.py 2>&1 | grep -E "^streaming \|mean\| in"
done
