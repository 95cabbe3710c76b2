set -e
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r3b_full_tests.log 2>&1
timeout -k 10 200 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r3b_smoke.log 2>&1
bash tools/side_configs.sh r3b
timeout -k 10 200 python3 tools/prefill_bench.py > gpurun_out/r3b_prefill.txt 2>&1
