#!/bin/bash
# diagnostic: 2 shard ranks on one GPU at C4 shape (small), collectives traced
cd $GRAFT_REPO_ROOT
python3 -c "import sys; sys.path.insert(0,'kube-batch-1_amd'); import kbgen; kbgen.gen_c4('/tmp/c4d.kbs', n_nodes=int(sys.argv[1]), n_pending=int(sys.argv[2]))" $1 $2
rm -f /tmp/dbg_init
for r in 0 1; do
  KBHIP_TRACE_SHARD=1 timeout -k 5 $3 python3 tests/shard_worker.py /tmp/c4d.kbs $r 2 /tmp/dbg_init gpurun_out/dbg_out$r.json allocate 1 > gpurun_out/dbg_rank$r.log 2>&1 &
done
wait
tail -3 gpurun_out/dbg_rank0.log gpurun_out/dbg_rank1.log
