#!/bin/bash
# r04 final probes on one MI355X (after the GPU suite and the bench pass):
# the standalone sweep, C3 and C5-allocate path counters (+ rocprofv3 of C3),
# placement-7 phases (stamps build), carry-over, the per-pop ABI host loops,
# C5 alone and 16 in flight (grouped and not), the shard rehearsal.
set -o pipefail
TAG=${1:-r04f}
export TMPDIR=/tmp
mkdir -p gpurun_out/$TAG
timeout -k 10 300 python -u profiles/sweep_probe.py 512 > gpurun_out/$TAG/sweep_probe.json 2> gpurun_out/$TAG/sweep_probe.err || exit 1
cat gpurun_out/$TAG/sweep_probe.json
timeout -k 10 300 python -u profiles/c3_probe.py 3 > gpurun_out/$TAG/c3_probe.json 2> gpurun_out/$TAG/c3.err || exit 1
cat gpurun_out/$TAG/c3_probe.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/$TAG/c3trace -o run --output-format csv -- \
    python3 profiles/c3_probe.py 1 > gpurun_out/$TAG/c3_trace.json 2> gpurun_out/$TAG/c3_trace.err || exit 1
cp gpurun_out/$TAG/c3trace/run_kernel_stats.csv gpurun_out/$TAG/c3_kernel_stats.csv
rm -rf gpurun_out/$TAG/c3trace
timeout -k 10 400 python -u profiles/c3_probe.py 2 --c5 > gpurun_out/$TAG/c5_alloc_probe.json 2> gpurun_out/$TAG/c5.err || exit 1
cat gpurun_out/$TAG/c5_alloc_probe.json
KBHIP_LIB=kube-batch-1_amd/_build/libkbhip_stamps.so timeout -k 10 300 python -u profiles/aff_phases.py 20000 \
    > gpurun_out/$TAG/aff_phases.json 2> gpurun_out/$TAG/aff_phases.err || exit 1
cat gpurun_out/$TAG/aff_phases.json
KBHIP_OPEN_PROFILE=1 timeout -k 10 400 python -u bench_carry.py --rounds 3 > gpurun_out/$TAG/carry.json 2> gpurun_out/$TAG/carry.err || exit 1
cat gpurun_out/$TAG/carry.json
grep "^\[carry\]" gpurun_out/$TAG/carry.err | tail -12 > gpurun_out/$TAG/carry_phases.txt
bash profiles/r04_host.sh $TAG || exit 1
SKIP_TESTS=1 bash profiles/r04_shard.sh $TAG || exit 1
