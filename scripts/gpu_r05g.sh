#!/bin/bash
# Round 5: decoder attention tests, asm-vs-builtin transposed LDS reads A/B, val-Dice with the per-pair HIP column.
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${TAG:-r05g}; mkdir -p $O; cd $R
timeout -k 10 300 python -u -m pytest -v -s --timeout 120 --timeout-method thread tests/test_gpu_dec_attn.py \
  > $O/dec_attn.log 2>&1; rc=$?
grep "rel-Frob\|passed\|failed" $O/dec_attn.log | cut -c1-330
[ $rc -gt 1 ] && exit $rc
for rnd in 1 2; do
  timeout -k 10 200 python -u scripts/dec_attn_ab.py run asm$rnd > $O/dab_asm$rnd.log 2>&1 || { tail -5 $O/dab_asm$rnd.log; exit 1; }
  OCTSAM_LIB=$R/ab_libs/liboctsam_dec_builtin.so timeout -k 10 200 python -u scripts/dec_attn_ab.py run bi$rnd > $O/dab_bi$rnd.log 2>&1 || { tail -5 $O/dab_bi$rnd.log; exit 1; }
done
python scripts/dec_attn_ab.py cmp asm1 bi1; python scripts/dec_attn_ab.py cmp asm2 bi2
OCTSAM_VALDICE_HIP_OUT=$O/valdice_hip.json timeout -k 10 900 python -u -m pytest -x -v -s --timeout 880 \
  --timeout-method thread tests/test_gpu_val_dice.py > $O/valdice.log 2>&1; rc=$?
tail -4 $O/valdice.log
cat $O/valdice_hip.json | head -60
exit $rc
