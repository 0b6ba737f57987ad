"""Full-size parity of the headline configs (BASELINE.json C4, and C3 with a
required-affinity / inter-pod-priority variant).

The engine's placement log on the exact bench snapshot must equal the CPU
oracle's, bit for bit.  The oracle's logs are pinned as digests in
tests/golden/fullsize.json (tests/golden/make_fullsize.py: oracle/kbfast.cpp on
the same kbgen snapshot); the snapshot digest pins the generator.  Running the
oracle live at these sizes takes minutes of host time, so the digest is the
checker here; tests/test_golden.py re-derives the snapshot digests on CPU.
"""
import hashlib
import json
import os

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = json.load(open(os.path.join(HERE, "golden", "fullsize.json")))

pytestmark = pytest.mark.gpu


def _digest(pod, node, kind):
    status = np.where(np.asarray(kind) == 1, 4, 8)
    return hashlib.sha256(np.stack([pod, node, status]).astype(np.int32).tobytes()).hexdigest()


def _check(engine, path, gold, **opts):
    with engine.Session(path) as s:
        for k, v in opts.items():
            s.set_option(k, v)
        pod, node, kind = s.allocate(cap=1 << 21)
    head = [[int(a), int(b), 4 if k == 1 else 8] for a, b, k in zip(pod[:64], node[:64], kind[:64])]
    assert head == gold["head"][: len(head)]
    assert len(pod) == gold["n"]
    assert _digest(pod, node, kind) == gold["log_sha256"]


@pytest.mark.skipif("c4" not in GOLD, reason="no C4 digest")
def test_c4_full_size_parity(engine, kbgen_mod, tmp_path):
    """C4: 100k nodes x 1M pods (200k running, 800k pending) — the bench's snapshot."""
    p = str(tmp_path / "c4.kbs")
    kbgen_mod.gen_c4(p)
    with open(p, "rb") as f:
        assert hashlib.sha256(f.read()).hexdigest() == GOLD["c4"]["snap_sha256"]
    _check(engine, p, GOLD["c4"])


@pytest.mark.skipif("c3" not in GOLD, reason="no C3 digest")
def test_c3_full_size_parity(engine, kbgen_mod, tmp_path):
    """C3: 20k nodes, labels / taints / selectors, zone anti-affinity, 8 queues."""
    p = str(tmp_path / "c3.kbs")
    kbgen_mod.gen_c3().write(p)
    with open(p, "rb") as f:
        assert hashlib.sha256(f.read()).hexdigest() == GOLD["c3"]["snap_sha256"]
    _check(engine, p, GOLD["c3"])


@pytest.mark.skipif("c3aff" not in GOLD, reason="no C3 affinity digest")
def test_c3_affinity_ipa_full_size_parity(engine, kbgen_mod, tmp_path):
    """C3 at full size with keyless nodes, required pod affinity and preferred
    inter-pod affinity / anti-affinity terms beside its zone anti-affinity
    (make_fullsize.py C3AFF; predicates.go:1402-1458, interpod_affinity.go:119-240)."""
    p = str(tmp_path / "c3aff.kbs")
    kbgen_mod.gen_c3(keyless=0.1, pod_affinity=0.15, ipa=0.15).write(p)
    with open(p, "rb") as f:
        assert hashlib.sha256(f.read()).hexdigest() == GOLD["c3aff"]["snap_sha256"]
    _check(engine, p, GOLD["c3aff"])
