"""One rank of a sharded allocate session (spawned by tests): opens the shard
of the snapshot on GPU 0 (ranks share the card), exchanges over gloo, runs the
given actions and writes the placement log as JSON.

usage: shard_worker.py <snapshot> <rank> <world> <init_file> <out.json> <actions> [batched]
(batched 1, default: the per-pop all-gather path is connected; 0: per-task only)
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kube-batch-1_amd"))


def main():
    import faulthandler  # a rank stuck for minutes prints where (the test's timeout then ends it)
    faulthandler.dump_traceback_later(120, repeat=True)
    path, rank, world, init_file, out, actions = sys.argv[1:7]
    batched = int(sys.argv[7]) if len(sys.argv) > 7 else 1
    rank, world = int(rank), int(world)
    import torch.distributed as dist
    import kbhip
    dist.init_process_group("gloo", init_method=f"file://{init_file}", rank=rank, world_size=world)
    import time
    t0 = time.time()

    def mark(what):  # progress on stderr: a slow or stuck rank shows where
        print(f"rank {rank}/{world}: {what} at {time.time() - t0:.1f} s", file=sys.stderr, flush=True)
    mark("process group formed")
    with kbhip.ShardedSession(path, 0, rank, world) as s:
        mark("session open")
        exchange = os.environ.get("KBHIP_TEST_EXCHANGE", "host")
        if exchange.endswith("_cu"):  # this rank's streams on its own share of the CUs (option cu_split)
            exchange = exchange[:-3]
            s.set_option("cu_split", rank * 256 + world)
        s.connect_host(kbhip.torch_exchange(), kbhip.torch_gather() if batched and exchange == "host" else None)
        if batched and exchange in ("mailbox", "mailbox_serial"):  # batched pops through the peer mailboxes
            s.connect_mailbox(kbhip.torch_gather())
            # "mailbox": a shard's sweep of pop e beside pop e-1's placement (the default);
            # "mailbox_serial": sweep, exchange and placement one after another
            s.set_option("shard_overlap", 0 if exchange == "mailbox_serial" else 1)
        info = s.info()
        pod, node, kind = s.run_actions(actions)
        if os.environ.get("KBHIP_TEST_CARRY") is not None:  # carry over (deleting the listed pods), run again
            dels = [int(x) for x in os.environ["KBHIP_TEST_CARRY"].split(",") if x]
            s.carry_events(dels, [1] * len(dels))
            pod, node, kind = s.run_actions(actions)
        mark("actions done")
        st = s.stats()
        close = s.gang_unschedulable()
    dist.barrier()
    dist.destroy_process_group()
    import hashlib

    import numpy as np
    status = np.where(np.asarray(kind) == 1, 4, 8)
    digest = hashlib.sha256(np.stack([pod, node, status]).astype(np.int32).tobytes()).hexdigest()
    full = os.environ.get("KBHIP_TEST_DIGEST_ONLY") is None
    with open(out, "w") as f:
        json.dump({"info": info, "n": int(len(pod)), "log_sha256": digest,
                   "head": [[int(a), int(b), int(k)] for a, b, k in zip(pod[:64], node[:64], kind[:64])],
                   "log": [[int(a), int(b), int(k)] for a, b, k in zip(pod, node, kind)] if full else None,
                   "batched_pops": st["batched_pops"], "sweeps": st["sweeps"], "collectives": st["collectives"],
                   "close": close}, f)


if __name__ == "__main__":
    main()
