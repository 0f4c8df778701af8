export TMPDIR=/tmp
set -e
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
timeout -k 10 200 python bench.py --workload symmetric --size 16384 --no-cpu > gpurun_out/bench_sym_n16384.json 2>/dev/null
timeout -k 10 200 python bench.py --workload symmetric --no-cpu > gpurun_out/bench_sym_n65536.json 2>/dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_sym -o sym --output-format csv -- python3 bench.py --workload symmetric --no-cpu --steps 20 > gpurun_out/bench_sym_rocprof.json 2>/dev/null
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_sym_f -o f --output-format csv -- python3 bench.py --workload symmetric --no-cpu --steps 4 --warmup 1 > /dev/null 2>&1
timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_sym_w -o w --output-format csv -- python3 bench.py --workload symmetric --no-cpu --steps 4 --warmup 1 > /dev/null 2>&1
for f in gpurun_out/bench_sym_n16384.json gpurun_out/bench_sym_n65536.json; do python3 -c "import json;d=json.load(open('$f'));print(d['config']['n'],'it/s %.1f'%d['value'],'mv_ms %.4f'%d['matvec_ms'],'GB/s %.0f'%d['matvec_gbps'],'relres',d['check']['relres'])"; done
