"""One rank of the CPU exchange test: reduces fixed per-rank values with
kbhip.torch_exchange over gloo and writes the results as JSON.

usage: exchange_worker.py <rank> <world> <init_file> <out.json>
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kube-batch-1_amd"))


def values(rank):
    # u64 keys: (score ^ 2^31) << 32 | (0x7fffffff - idx) << 1 | kind  (top bit set for score >= 0)
    keys = np.array([(((s ^ 0x80000000) & 0xffffffff) << 32) | ((0x7fffffff - i) << 1) | k
                     for s, i, k in [(3 + rank, 10 * rank, 0), (-2, rank, 1), (0, 5 - rank, 0)]], dtype=np.uint64)
    return keys, np.array([-7 * rank, 4 - rank], dtype=np.int64)


def main():
    rank, world, init_file, out = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3], sys.argv[4]
    import torch.distributed as dist
    import kbhip
    dist.init_process_group("gloo", init_method=f"file://{init_file}", rank=rank, world_size=world)
    fn = kbhip.torch_exchange()
    keys, ints = values(rank)
    res = {"max_u64": [], "min_i64": [], "max_i64": [], "sum_i64": []}
    for k in keys:
        v = np.array([k], dtype=np.uint64)
        fn(v, kbhip.RED_MAX_U64)
        res["max_u64"].append(int(v[0]))
    for x in ints:
        v = np.array([x], dtype=np.int64).view(np.uint64)
        fn(v, kbhip.RED_MIN_I64)
        res["min_i64"].append(int(v.view(np.int64)[0]))
        v = np.array([x], dtype=np.int64).view(np.uint64)
        fn(v, kbhip.RED_MAX_I64)
        res["max_i64"].append(int(v.view(np.int64)[0]))
    # several values per call, summed (the FitDelta counts of a walk over the shards)
    v = ints.copy().view(np.uint64)
    fn(v, kbhip.RED_SUM_I64)
    res["sum_i64"] = [int(x) for x in v.view(np.int64)]
    # all-gather of a per-rank byte record (the batched shard path's ShardMsg exchange)
    g = kbhip.torch_gather()
    send = (np.arange(40, dtype=np.uint8) * (rank + 1)).astype(np.uint8)
    recv = np.zeros(40 * world, dtype=np.uint8)
    g(send, recv)
    res["gather"] = [int(x) for x in recv]
    dist.destroy_process_group()
    with open(out, "w") as f:
        json.dump(res, f)


if __name__ == "__main__":
    main()
