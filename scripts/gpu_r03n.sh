#!/bin/bash
# rocprofv3 kernel traces: the default bench command (pipelined, the bench line's own profile) and the sequential
# step (--pipeline 0), each reduced to the stats CSV + a compact per-kernel table (trace CSVs deleted).
set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${TAG:-r03n}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $O/seq -o run -- python3 $R/bench.py --pipeline 0 --cpu-baseline 0 --val 0 --topo-all 0 > $O/seq.log 2>&1 || { tail -5 $O/seq.log; exit 1; }
python3 $R/scripts/prof_summary.py $O/seq $O/seq_kernels.csv --delete-trace || exit 1
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/pipe -o run -- python3 $R/bench.py > $O/pipe.log 2>&1 || { tail -5 $O/pipe.log; exit 1; }
python3 $R/scripts/prof_summary.py $O/pipe $O/pipe_kernels.csv --delete-trace || exit 1
grep -h '"metric"' $O/pipe.log | cut -c1-300
find $O -name "*.csv" | head; du -sh $O
