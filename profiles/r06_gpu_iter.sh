# Round-6 iteration run: engine tests (list + sweep mode), then the C4 bench.
set -o pipefail
mkdir -p gpurun_out
tag=${1:-r06b}
timeout -k 10 600 python -u -m pytest tests/test_gpu_engine.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${tag}_engine_tests.log 2>&1 && \
timeout -k 10 300 python -u bench.py > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err
