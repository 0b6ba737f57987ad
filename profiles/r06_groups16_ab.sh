# More merger groups (KBHIP_ENG_GROUPS=16 build, _build/libkbhip_g16.so, loaded
# (the g16 build came from a patch not kept: the final merger looping over group lists
# wave, wave + 8 and a KBHIP_ENG_GROUPS build knob)
# with KBHIP_LIB): its engine parity suites, then the bench alternating the
# product (8 groups) with 16 and 12 groups on one box.
set -o pipefail
mkdir -p gpurun_out
KBHIP_LIB=$PWD/kube-batch-1_amd/_build/libkbhip_g16.so timeout -k 10 600 python3 -u -m pytest tests/test_gpu_engine.py tests/test_gpu_multiblock.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r06g16_pytest.log 2>&1 || { tail -30 gpurun_out/r06g16_pytest.log; exit 1; }
tail -1 gpurun_out/r06g16_pytest.log
for v in p8 g16 g12 p8 g16 g12; do
  case $v in
    p8) unset KBHIP_LIB; G=-1 ;;
    g16) export KBHIP_LIB=$PWD/kube-batch-1_amd/_build/libkbhip_g16.so; G=-1 ;;
    g12) export KBHIP_LIB=$PWD/kube-batch-1_amd/_build/libkbhip_g16.so; G=12 ;;
  esac
  timeout -k 10 300 python3 -u bench.py --steps 8 --warmup 2 --cpu-baseline 0 --sweep-nodes 0 --engine-groups $G > gpurun_out/r06g16_$v.json 2> gpurun_out/r06g16_$v.err || { tail -20 gpurun_out/r06g16_$v.err; exit 1; }
  python3 -c "import json;d=json.loads(open('gpurun_out/r06g16_$v.json').read().strip().splitlines()[-1]);c=d['config'];print('$v', round(d['value']), round(d['p50_session_ms'],1), round(c['device_period_us'],3), c['engine_pops'], c['engine_workers'])"
done
