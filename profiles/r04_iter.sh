#!/bin/bash
# r04 iteration: parity of the changed paths, then the probes and a short bench.
set -o pipefail
TAG=${1:-r04i}
export TMPDIR=/tmp
mkdir -p gpurun_out/$TAG
timeout -k 10 800 python -u -m pytest tests/test_gpu_aff_batch.py tests/test_gpu_fullsize.py::test_c3_full_size_parity \
    tests/test_gpu_async_abi.py tests/test_gpu_carry_snapshot.py tests/test_gpu_carry.py -x -q --timeout 300 \
    --timeout-method thread > gpurun_out/$TAG/pytest.log 2>&1 || { tail -40 gpurun_out/$TAG/pytest.log; exit 1; }
tail -1 gpurun_out/$TAG/pytest.log
KBHIP_LIB=kube-batch-1_amd/_build/libkbhip_stamps.so timeout -k 10 300 python -u profiles/aff_phases.py 20000 \
    > gpurun_out/$TAG/aff_phases.json 2> gpurun_out/$TAG/aff_phases.err || { tail -20 gpurun_out/$TAG/aff_phases.err; exit 1; }
cat gpurun_out/$TAG/aff_phases.json
timeout -k 10 300 python -u profiles/c3_probe.py 3 > gpurun_out/$TAG/c3.json 2> gpurun_out/$TAG/c3.err || exit 1
cat gpurun_out/$TAG/c3.json
KBHIP_OPEN_PROFILE=1 timeout -k 10 400 python -u bench_carry.py --rounds 2 > gpurun_out/$TAG/carry.json 2> gpurun_out/$TAG/carry.err || { tail -20 gpurun_out/$TAG/carry.err; exit 1; }
cat gpurun_out/$TAG/carry.json
grep "^\[carry\]" gpurun_out/$TAG/carry.err | tail -8
timeout -k 10 600 python -u bench.py --steps 10 --warmup 3 > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err || { tail -20 gpurun_out/$TAG/bench.err; exit 1; }
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print({k: d[k] for k in ('value','ms_per_step','p50_session_ms')}, d['config']['device_period_us'], d['roofline']['frac'])" gpurun_out/$TAG/bench.json
