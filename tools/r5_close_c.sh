#!/bin/bash
# Round-5 close, part C: the kernel-trace pass of part B alone (re-run after part B's trace faulted without
# DEBUG_CLR_GRAPH_PACKET_CAPTURE=0).
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/close
mkdir -p $O
DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline \
  > $O/prof_bench.json 2> $O/prof.err || { grep -v '^    @' $O/prof.err | tail -20; exit 1; }
DB=$(ls $O/prof/run_results.db $O/prof/*/run_results.db 2>/dev/null | head -1)
python3 tools/rocpd_summary.py $DB > $O/bench_kernel_stats.txt && python3 tools/roofline_from_trace.py $DB > $O/roofline_from_trace.txt || exit 1
head -8 $O/bench_kernel_stats.txt; cat $O/roofline_from_trace.txt; cat $O/prof_bench.json | cut -c1-300
rm -rf $O/prof
