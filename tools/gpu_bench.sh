# the round's bench lines: default, then --extras
set -u
O=gpurun_out/${1:-r06_bench}; mkdir -p $O
timeout -k 10 400 python3 bench.py > $O/bench.json 2> $O/bench.err || { echo bench failed; tail $O/bench.err; exit 1; }
timeout -k 10 600 python3 bench.py --extras > $O/bench_extras.json 2> $O/bench_extras.err || { echo extras failed; tail $O/bench_extras.err; exit 1; }
head -c 1500 $O/bench.json
