#!/bin/bash
# Round 4: persistence ranking by 32-bit persistence images + the position-major keys' weight gradient (octsam_wgrad_pe):
# bit-exactness / parity tests, PH phase timing, step A/B of wgrad_pe.
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${TAG:-r04p}; mkdir -p $O; cd $R
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_ph.py tests/test_gpu_topo_w2.py > $O/pytest_ph.log 2>&1 || { tail -30 $O/pytest_ph.log; exit 1; }
tail -1 $O/pytest_ph.log
timeout -k 10 60 ./scripts/micro/ph_timing_probe > $O/ph_timing.log 2>&1 || { tail -5 $O/ph_timing.log; exit 1; }
cat $O/ph_timing.log
timeout -k 10 60 ./scripts/micro/uf_resolve_probe > $O/uf_resolve_probe.log 2>&1 || exit 1
cat $O/uf_resolve_probe.log
timeout -k 10 400 python -u -m pytest -x -v --timeout 280 --timeout-method thread tests/test_gpu_dec_attn.py tests/test_gpu_gemm.py -k "wgrad or t2i or i2t or decoder or model" tests/test_gpu_model.py > $O/pytest_w.log 2>&1 || { tail -30 $O/pytest_w.log; exit 1; }
tail -1 $O/pytest_w.log
STEP_VARIANTS=default,pe_off,t2isum_off timeout -k 10 400 python -u scripts/step_ab3.py > $O/step_ab_pe.log 2>&1 || { tail -20 $O/step_ab_pe.log; exit 1; }
tail -1 $O/step_ab_pe.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/profseq -o run -- python3 $R/bench.py --pipeline 0 --cpu-baseline 0 --val 0 --val-protocol 0 --top-off 0 --data-path 0 --e2e-steps 0 --topo-all 0 --loop-images 0 > $O/profseq.log 2>&1 || { tail -5 $O/profseq.log; exit 1; }
python3 $R/scripts/prof_summary.py $O/profseq $O/kernel_stats_sequential.csv --delete-trace || exit 1
grep -E "cubical|wgrad_kernel|group_sum" $O/kernel_stats_sequential.csv | cut -c1-60,200-
