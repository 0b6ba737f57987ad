#!/bin/bash
# r04 probes on one MI355X: placement-7 phases (stamps build), the C3 and
# C5-allocate path counters, C5 under rocprofv3.
set -o pipefail
TAG=${1:-r04p}
export TMPDIR=/tmp
mkdir -p gpurun_out/$TAG
KBHIP_LIB=kube-batch-1_amd/_build/libkbhip_stamps.so timeout -k 10 300 python -u profiles/aff_phases.py 20000 \
    > gpurun_out/$TAG/aff_phases.json 2> gpurun_out/$TAG/aff_phases.err || { tail -20 gpurun_out/$TAG/aff_phases.err; exit 1; }
cat gpurun_out/$TAG/aff_phases.json
timeout -k 10 300 python -u profiles/c3_probe.py 3 > gpurun_out/$TAG/c3.json 2> gpurun_out/$TAG/c3.err || exit 1
cat gpurun_out/$TAG/c3.json
timeout -k 10 400 python -u profiles/c3_probe.py 2 --c5 > gpurun_out/$TAG/c5.json 2> gpurun_out/$TAG/c5.err || { tail -20 gpurun_out/$TAG/c5.err; exit 1; }
cat gpurun_out/$TAG/c5.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/$TAG/c5trace -o run --output-format csv -- \
    python3 profiles/c3_probe.py 1 --c5 > gpurun_out/$TAG/c5_trace.json 2> gpurun_out/$TAG/c5_trace.err || exit 1
cp gpurun_out/$TAG/c5trace/run_kernel_stats.csv gpurun_out/$TAG/c5_kernel_stats.csv
rm -rf gpurun_out/$TAG/c5trace
head -12 gpurun_out/$TAG/c5_kernel_stats.csv
