#!/bin/bash
# Round 4: windowed-attention rewrite check (tests + A/B of the idle-wave variants), smoke, the W2/PH/step-oracle/
# graph tests and a default bench line.
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${TAG:-r04c}; mkdir -p $O; cd $R
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_layers.py -k "vit_attention" > $O/pytest_attn.log 2>&1 || { tail -30 $O/pytest_attn.log; exit 1; }
tail -1 $O/pytest_attn.log
ATTN_VARIANTS=100,101 timeout -k 10 200 python -u scripts/attn_ab.py > $O/attn_ab.log 2>&1 || { tail -20 $O/attn_ab.log; exit 1; }
cat $O/attn_ab.log
timeout -k 10 400 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 600 python -u -m pytest -x -v --timeout 280 --timeout-method thread tests/test_gpu_topo_w2.py tests/test_gpu_ph.py tests/test_gpu_step_oracle.py tests/test_gpu_graph_step.py > $O/pytest_a.log 2>&1 || { tail -30 $O/pytest_a.log; exit 1; }
tail -1 $O/pytest_a.log
grep -E "DiceCE" $O/pytest_a.log || true
timeout -k 10 500 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cut -c1-400 $O/bench.json
