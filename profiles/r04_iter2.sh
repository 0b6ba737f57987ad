#!/bin/bash
# r04 iteration 2: allocate without the idle-job pops, placement-6 backoff,
# node task lists sized: parity of every allocate / evict path, then C5 / C3
# probes and a short C4 bench.
set -o pipefail
TAG=${1:-r04j}
export TMPDIR=/tmp
mkdir -p gpurun_out/$TAG
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_backfilled.py tests/test_gpu_evict.py \
    tests/test_gpu_whatif.py tests/test_gpu_async_abi.py tests/test_gpu_fullsize.py tests/test_gpu_aff_batch.py \
    tests/test_gpu_place_job.py tests/test_gpu_fit_error.py -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/$TAG/pytest.log 2>&1 || { tail -40 gpurun_out/$TAG/pytest.log; exit 1; }
tail -1 gpurun_out/$TAG/pytest.log
timeout -k 10 400 python -u bench_c5.py --concurrent 1 --sessions 5 --warmup 1 --cpu-baseline 0 > gpurun_out/$TAG/c5_alone.json 2> gpurun_out/$TAG/c5_alone.err || exit 1
cat gpurun_out/$TAG/c5_alone.json
timeout -k 10 400 python -u profiles/c3_probe.py 2 --c5 > gpurun_out/$TAG/c5.json 2> gpurun_out/$TAG/c5.err || { tail -20 gpurun_out/$TAG/c5.err; exit 1; }
cat gpurun_out/$TAG/c5.json
timeout -k 10 300 python -u profiles/c3_probe.py 3 > gpurun_out/$TAG/c3.json 2> gpurun_out/$TAG/c3.err || exit 1
cat gpurun_out/$TAG/c3.json
timeout -k 10 600 python -u bench.py --steps 10 --warmup 3 > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err || { tail -20 gpurun_out/$TAG/bench.err; exit 1; }
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print({k: d[k] for k in ('value','ms_per_step','p50_session_ms')}, d['config']['device_period_us'], d['config']['session_phases_ms'], d['roofline']['frac'])" gpurun_out/$TAG/bench.json
KBHIP_OPEN_PROFILE=1 timeout -k 10 400 python -u bench_carry.py --rounds 2 > gpurun_out/$TAG/carry.json 2> gpurun_out/$TAG/carry.err || { tail -20 gpurun_out/$TAG/carry.err; exit 1; }
cat gpurun_out/$TAG/carry.json
grep "^\[carry\]" gpurun_out/$TAG/carry.err | tail -12
