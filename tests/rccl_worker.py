"""One rank of a node-sharded session over RCCL (spawned by tests): rank r uses
GPU r; rank 0 writes the RCCL unique id to <init_file>.id, the others read it.

usage: rccl_worker.py <snapshot> <rank> <world> <init_file> <out.json>
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kube-batch-1_amd"))


def main():
    path, rank, world, init_file, out = sys.argv[1:6]
    rank, world = int(rank), int(world)
    import kbhip
    idf = init_file + ".id"
    if rank == 0:
        uid = kbhip.ShardedSession.rccl_unique_id()
        with open(idf + ".tmp", "wb") as f:
            f.write(uid)
        os.replace(idf + ".tmp", idf)
    else:
        for _ in range(600):
            if os.path.exists(idf):
                break
            time.sleep(0.1)
        with open(idf, "rb") as f:
            uid = f.read()
    with kbhip.ShardedSession(path, rank, rank, world) as s:
        s.connect_rccl(uid)
        pod, node, kind = s.run_actions("allocate, backfill")
    with open(out, "w") as f:
        json.dump({"log": [[int(a), int(b), int(k)] for a, b, k in zip(pod, node, kind)]}, f)


if __name__ == "__main__":
    main()
