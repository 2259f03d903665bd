#!/bin/bash
# Token-side weight gradients, two builds: parity tests, per-kernel time under rocprofv3 for both builds,
# same-box step A/B against ${LIB_B}.
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${TAG:-tokxcd}; mkdir -p $O; cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_gemm.py tests/test_gpu_model.py -m gpu -x -q -k "wgrad_tok or tok_group" --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
cd /tmp && export TMPDIR=/tmp
for lib in default ${LIB_B}; do
  if [ $lib = default ]; then unset OCTSAM_LIB; else export OCTSAM_LIB=$R/$lib; fi
  n=$(basename $lib)
  ROUNDS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$n -o run -- python3 $R/scripts/step_ab2.py 1:0 > $O/prof_$n.log 2>&1 || { tail -5 $O/prof_$n.log; exit 1; }
  python3 $R/scripts/prof_summary.py $O/prof_$n $O/stats_$n.csv --delete-trace > /dev/null || exit 1
  echo "$n: $(grep wgrad_tok_group $O/stats_$n.csv | cut -d, -f1-4 | tr '\n' ' ')"
done
unset OCTSAM_LIB
cd $R
TAG=${TAG}/step LIB_B=${LIB_B} bash scripts/step_lib_ab.sh
