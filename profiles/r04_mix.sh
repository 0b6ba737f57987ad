#!/bin/bash
# r04 iteration on one MI355X: affinity / speculation parity (placement 7 with
# per-domain candidates, the parallel undo), the C3 probe under rocprofv3, the
# carry-over phases (KBHIP_OPEN_PROFILE), the shard rehearsal.
# usage: bash profiles/r04_mix.sh TAG
set -o pipefail
TAG=${1:-r04m}
export TMPDIR=/tmp
mkdir -p gpurun_out/$TAG
timeout -k 10 800 python -u -m pytest tests/test_gpu_aff_batch.py tests/test_gpu_fullsize.py tests/test_gpu_async_abi.py \
    tests/test_gpu_parity.py tests/test_gpu_carry_snapshot.py -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/$TAG/pytest.log 2>&1 || { tail -40 gpurun_out/$TAG/pytest.log; exit 1; }
tail -1 gpurun_out/$TAG/pytest.log
timeout -k 10 300 python -u profiles/c3_probe.py 3 > gpurun_out/$TAG/c3.json 2> gpurun_out/$TAG/c3.err || exit 1
cat gpurun_out/$TAG/c3.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/$TAG/c3trace -o run --output-format csv -- \
    python3 profiles/c3_probe.py 1 > gpurun_out/$TAG/c3_trace.json 2> gpurun_out/$TAG/c3_trace.err || exit 1
cp gpurun_out/$TAG/c3trace/run_kernel_stats.csv gpurun_out/$TAG/c3_kernel_stats.csv
rm -rf gpurun_out/$TAG/c3trace
head -8 gpurun_out/$TAG/c3_kernel_stats.csv
KBHIP_OPEN_PROFILE=1 timeout -k 10 400 python -u bench_carry.py --rounds 2 > gpurun_out/$TAG/carry.json 2> gpurun_out/$TAG/carry.err || { tail -20 gpurun_out/$TAG/carry.err; exit 1; }
cat gpurun_out/$TAG/carry.json
grep "^\[carry\]" gpurun_out/$TAG/carry.err | tail -24
SKIP_TESTS=1 bash profiles/r04_shard.sh $TAG
