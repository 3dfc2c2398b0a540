set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > gpurun_out/t1.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --host-runs 3 > gpurun_out/b1.json 2> gpurun_out/b1.err
