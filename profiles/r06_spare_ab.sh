# A/B of the spare host pools on one box, alternating builds: C5 alone (and C4
# when C4=1): prev = no spare pools (_build/libkbhip_prev.so), u = job UIDs
# only (_build/libkbhip_u.so), cur = job records + UIDs (_build/libkbhip.so)
set -o pipefail
mkdir -p gpurun_out
for v in ${VARIANTS:-prev u cur prev u cur}; do
  case $v in
    prev) export KBHIP_LIB=$PWD/kube-batch-1_amd/_build/libkbhip_prev.so ;;
    u) export KBHIP_LIB=$PWD/kube-batch-1_amd/_build/libkbhip_u.so ;;
    *) unset KBHIP_LIB ;;
  esac
  timeout -k 10 300 python3 -u bench_c5.py --sessions 6 --warmup 1 --concurrent 1 --cpu-baseline 0 > gpurun_out/r06q_c5_$v.json 2> gpurun_out/r06q_c5_$v.err || { tail -20 gpurun_out/r06q_c5_$v.err; exit 1; }
  python3 -c "import json,sys;d=json.loads(open('gpurun_out/r06q_c5_$v.json').read().strip().splitlines()[-1]);print('$v c5', round(d['p50_session_ms'],1), d['phases_ms'])"
  if [ "${C4:-0}" = 1 ]; then
    timeout -k 10 300 python3 -u bench.py --steps 8 --warmup 2 --cpu-baseline 0 --sweep-nodes 0 > gpurun_out/r06q_c4_$v.json 2> gpurun_out/r06q_c4_$v.err || { tail -20 gpurun_out/r06q_c4_$v.err; exit 1; }
    python3 -c "import json,sys;d=json.loads(open('gpurun_out/r06q_c4_$v.json').read().strip().splitlines()[-1]);print('$v c4', round(d['value']), round(d['p50_session_ms'],1), d['config']['session_phases_ms'])"
  fi
done
