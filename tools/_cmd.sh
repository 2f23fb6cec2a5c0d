set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/cfg
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/cfg/tests.log 2>&1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/cfg/smoke.log 2>&1
timeout -k 10 200 python bench.py --config 1 --no-cpu-baseline --alt-ans-streams 0 > gpurun_out/cfg/bench_4k.log 2>&1
timeout -k 10 200 python bench.py --config 4 --proposals 3 --steps 4 --warmup 1 --no-cpu-baseline --alt-ans-streams 0 > gpurun_out/cfg/bench_16k_pf.log 2>&1
timeout -k 10 200 python bench.py --config 2 --proposals 3 --no-cpu-baseline --alt-ans-streams 0 > gpurun_out/cfg/bench_8k_pf.log 2>&1
timeout -k 10 200 python bench.py --coder ans --streams 3 --no-cpu-baseline --alt-ans-streams 0 > gpurun_out/cfg/bench_8k_ans3.log 2>&1
