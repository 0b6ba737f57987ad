#!/bin/bash
# r03 measurements of HEAD on one MI355X: per-pop ABI at C4 (kbhost, sync and
# async), C5 what-if group (lockstep on / off), rocprofv3 of the C4 bench.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u profiles/host_loop.py --reps 3 --depth 2 --out gpurun_out/r03_host_loop.json \
    > gpurun_out/r03_host_loop.log 2>&1 || exit $?
timeout -k 10 300 python -u bench_c5.py --sessions 16 --concurrent 8 --group 1 --cpu-baseline 0 \
    > gpurun_out/r03_c5_group1.json 2> gpurun_out/r03_c5_group1.err || exit $?
timeout -k 10 300 python -u bench_c5.py --sessions 16 --concurrent 8 --group 0 --cpu-baseline 0 \
    > gpurun_out/r03_c5_group0.json 2> gpurun_out/r03_c5_group0.err || exit $?
bash profiles/run_profile.sh r03a > gpurun_out/r03_prof.log 2>&1 || exit $?
