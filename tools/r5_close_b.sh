#!/bin/bash
# Round-5 close, part B: the default bench line, the side configurations, the 512-token prefill, and a
# rocprofv3 kernel trace of the default bench summarised on the box (per-kernel stats, roofline by step position;
# DEBUG_CLR_GRAPH_PACKET_CAPTURE=0: the kernel tracer faults inside hipGraphLaunch without it).
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/close
mkdir -p $O
timeout -k 10 300 python3 bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
bash tools/side_configs.sh close || exit 1
mv gpurun_out/close_side.jsonl $O/side.jsonl
timeout -k 10 200 python3 tools/prefill_bench.py 512 > $O/prefill.txt 2>&1 || { tail -20 $O/prefill.txt; exit 1; }
cat $O/prefill.txt
DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline \
  > $O/prof_bench.json 2> $O/prof.err || { tail -20 $O/prof.err; exit 1; }
DB=$(ls $O/prof/run_results.db $O/prof/*/run_results.db 2>/dev/null | head -1)
python3 tools/rocpd_summary.py $DB > $O/bench_kernel_stats.txt && python3 tools/roofline_from_trace.py $DB > $O/roofline_from_trace.txt || exit 1
head -8 $O/bench_kernel_stats.txt; cat $O/roofline_from_trace.txt
rm -rf $O/prof
