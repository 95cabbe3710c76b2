set -e
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python3 $R/bench.py > $R/gpurun_out/r1_bench_final.json 2> $R/gpurun_out/r1_bench_final.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_stats -o run -- python3 $R/bench.py --steps 64 --warmup 4 --no-cpu-baseline --kernel-reps 20 > $R/gpurun_out/prof_stats.log 2>&1
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/pmc -o run -- python3 $R/bench.py --steps 4 --warmup 2 --kernel-reps 4 --no-cpu-baseline > $R/gpurun_out/pmc.log 2>&1
