#!/bin/bash
# r04 final pass A: the carry suites + carry bench (phase marks), the GPU suite,
# the C4 bench line with its rocprofv3 kernel stats and counter passes.
set -o pipefail
bash profiles/r04_carry2.sh r04fk || exit 1
bash profiles/r04_measure.sh r04final 1 || exit 1
