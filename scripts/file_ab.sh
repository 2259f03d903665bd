# Same-box two-build A/B: TESTS, then the pipelined step with the current lib vs build/ab/liboctsam_old.so
# (scripts/build_ab_lib.sh). usage: TAG=x TESTS="tests/a.py" bash scripts/file_ab.sh
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${TAG:-libab2}; mkdir -p $O; cd $R
timeout -k 10 400 python -u -m pytest ${TESTS} -x -q --timeout 120 --timeout-method thread > $O/t.log 2>&1 || { tail -5 $O/t.log; exit 1; }
tail -1 $O/t.log
for r in 1 2; do
  for lib in new old; do
    if [ $lib = old ]; then export OCTSAM_LIB=$R/dilabhelmholtzoct_amd/csrc/build/ab/liboctsam_old.so; else unset OCTSAM_LIB; fi
    ROUNDS=2 timeout -k 10 300 python scripts/step_ab2.py 1:1 > $O/st_${r}_$lib.log 2>&1 || exit 1
    echo "$lib round $r: $(tail -1 $O/st_${r}_$lib.log)"
  done
done
