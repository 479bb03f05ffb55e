# Path-4 kernel trace of single html uncompress calls + tools/small_check.py (design tool; GPU box)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/small_prof
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/small_prof/prof -o run -- python3 tools/small_prof.py html 30 > gpurun_out/small_prof/prof.log 2>&1 || { echo prof failed; tail gpurun_out/small_prof/prof.log; exit 1; }
find gpurun_out/small_prof/prof -name "*kernel_stats.csv" | head -1 | xargs cat | cut -d, -f1-4
timeout -k 10 200 python3 tools/small_check.py > gpurun_out/small_prof/small.log 2>&1; echo "small rc $?"; tail -8 gpurun_out/small_prof/small.log
