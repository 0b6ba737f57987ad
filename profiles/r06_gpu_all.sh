# Round-6 iteration: engine tests, list-mode timeline, C4 bench (list mode default)
set -o pipefail
mkdir -p gpurun_out
tag=${1:-r06x}
timeout -k 10 600 python -u -m pytest tests/test_gpu_engine.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${tag}_engine_tests.log 2>&1 && \
timeout -k 10 300 python -u profiles/engine_tl_lists.py --out gpurun_out/${tag}_tl_lists.json > gpurun_out/${tag}_tl.log 2>&1 && \
timeout -k 10 300 python -u bench.py > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err
