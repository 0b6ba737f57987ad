"""The per-pop boundary (kbhip_place_job, include/kbhip.h) driven the way the
Go shim of INTEGRATION.md drives it: the host keeps the reference's ordering
(allocate.go:41-201 with priority / gang / drf / proportion and Go's
container/heap, tests/gohost.py) and hands each job pop to the engine.  The
resulting placement log must equal the CPU oracle's, bit for bit; C2 also
reports the pop-at-a-time rate (the timing line of the per-pop ABI, written
to gpurun_out/place_job_c2.json when that directory exists)."""
import json
import os
import time

import pytest

from gohost import GoHost
from test_gpu_parity import NO_POD_AFFINITY

pytestmark = pytest.mark.gpu

TIERS = [None, [["drf", "proportion"]], [["gang"], ["predicates", "nodeorder"]],
         [["priority", "gang", "drf"], ["predicates", "proportion", "nodeorder", "nodeorder"]]]


def _drive(engine, path, cluster, **opts):
    with engine.Session(path) as s:
        for k, v in opts.items():
            s.set_option(k, v)

        def place_job(ids, gm, min_avail, ready):
            return s.place_job(ids, gm, min_avail, ready)
        t0 = time.perf_counter()
        log, pops = GoHost(cluster).allocate(place_job)
        return log, pops, time.perf_counter() - t0, s.stats()


@pytest.mark.parametrize("seed", range(24))
def test_place_job_host_loop_random(engine, oracle_mod, kbgen_mod, tmp_path, seed):
    feats = NO_POD_AFFINITY if seed % 3 else ("labels", "taints", "ports", "affinity", "init", "running",
                                              "releasing", "selector", "nodeaffinity", "podaffinity", "unsched")
    c = kbgen_mod.gen_random(9100 + seed, n_nodes=4 + seed % 12, n_jobs=4 + seed % 8, max_tasks=1 + seed % 8,
                             features=feats, tiers=TIERS[seed % 4], n_queues=1 + seed % 3)
    p = str(tmp_path / "r.kbs")
    c.write(p)
    exp = oracle_mod.ref_allocate(p).as_list()
    for opts in (dict(), dict(overlap=0), dict(batched=0)):
        got, _, _, _ = _drive(engine, p, c, **opts)
        assert got == exp, opts


def test_place_job_host_loop_c2(engine, oracle_mod, kbgen_mod, tmp_path):
    """C2 at full size (5k nodes x 50k pods) through the per-pop ABI."""
    p = str(tmp_path / "c2.kbs")
    kbgen_mod.gen_c2(p)
    exp = oracle_mod.fast_allocate(p, threads=16).as_list()
    c = kbgen_mod.cluster_from_kbs(p)  # the bulk generator writes columns: the object model read back
    got, pops, secs, st = _drive(engine, p, c)
    assert got == exp
    rec = {"config": "C2 5k nodes x 50k pods", "placements": len(got), "pops": pops, "seconds": secs,
           "placements_per_s": len(got) / secs, "batched_pops": st["batched_pops"],
           "host_loop": "tests/gohost.py (Python mirror of allocate.go:41-201) + kbhip_place_job per pop"}
    out = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gpurun_out")
    if os.path.isdir(out):
        with open(os.path.join(out, "place_job_c2.json"), "w") as f:
            json.dump(rec, f)
    print(json.dumps(rec))
