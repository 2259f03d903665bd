cd $GRAFT_REPO_ROOT
for f in 1 10 5 2; do
  for shape in "655360 256 256 0 0 0" "655360 128 256 0 0 0" "655360 256 128 0 1 1" "2621440 128 64 2 0 0" "655360 256 384 0 1 1"; do
    FAST=$f timeout -k 5 60 python scripts/gemm_probe.py $shape 10 2>&1 | grep fast= || exit 1
  done
done
