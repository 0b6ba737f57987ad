# Round-6: engine tests + the multi-block / keyless / hardened-C3 parity tests
set -o pipefail
mkdir -p gpurun_out
tag=${1:-r06q}
timeout -k 10 900 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_multiblock.py -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1
