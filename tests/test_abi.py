"""The C ABI library builds for gfx950, loads, and exports exactly what
include/kbhip.h declares (no compute calls here: this runs without a GPU)."""
import ctypes
import os
import re

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


def _declared():
    src = open(os.path.join(ROOT, "include", "kbhip.h")).read()
    return sorted(set(re.findall(r"\b(kbhip_[a-z_]+)\s*\(", src)))


def test_header_declares_abi():
    import kbhip
    assert set(_declared()) == set(kbhip.EXPORTS)


def test_library_exports_every_symbol(engine_lib):
    for name in _declared():
        assert hasattr(engine_lib, name), name


def test_library_contains_gfx950_code_object():
    import kbhip
    data = open(kbhip.LIB_PATH, "rb").read()
    assert b"gfx950" in data


def test_no_device_is_an_error_not_a_fallback(engine_lib):
    """Without a usable gfx950 device every session open fails loudly."""
    import kbhip
    n = engine_lib.kbhip_device_count()
    if n >= 1:
        return  # on the GPU box this is covered by the gpu tests
    h = ctypes.c_void_p()
    rc = engine_lib.kbhip_session_open_file(os.path.join(HERE, "golden", "c1_default.kbs").encode(), 0,
                                            ctypes.byref(h))
    assert rc == -2  # KBHIP_ENODEV


def test_score_outside_int32_rejected(engine_lib, tmp_path):
    """nodeorder weights whose score range leaves int32 (Go sums in 64-bit int,
    nodeorder.go:209-246, 287-313) are refused with KBHIP_EUNSUPPORTED, not
    silently wrapped."""
    import kbgen
    import kbhip
    for w in ("3000000000", "300000000"):
        c = kbgen.gen_c1()
        c.args = {"nodeorder": {"leastrequested.weight": w}}
        p = str(tmp_path / f"w{w}.kbs")
        c.write(p)
        with pytest.raises(kbhip.KbhipError, match="int32"):
            kbhip.EncodedSnapshot(p)
    c = kbgen.gen_c1()
    c.args = {"nodeorder": {"leastrequested.weight": "30000000"}}  # 10 x 3e7 fits
    p = str(tmp_path / "ok.kbs")
    c.write(p)
    kbhip.EncodedSnapshot(p).close()


def test_log_actions_validate_outputs(engine_lib):
    """A null session or null output arrays with cap > 0 return KBHIP_EINVAL."""
    import ctypes
    L = engine_lib
    for fn in (L.kbhip_allocate, L.kbhip_backfill, L.kbhip_reclaim, L.kbhip_preempt):
        assert fn(None, None, None, None, 4) == -1


def test_header_constants_match_binding():
    """Cache-event codes, placement kinds and stop reasons: the values the
    Python binding passes are the header's."""
    import kbhip
    src = open(os.path.join(ROOT, "include", "kbhip.h")).read()
    enum = dict(re.findall(r"\b(KBHIP_EV_[A-Z]+)\s*=\s*(\d+)", src))
    assert {k: int(v) for k, v in enum.items()} == {"KBHIP_EV_DELETE": kbhip.EV_DELETE,
                                                    "KBHIP_EV_SUCCEEDED": kbhip.EV_SUCCEEDED,
                                                    "KBHIP_EV_FAILED": kbhip.EV_FAILED}
    defs = {k: int(v) for k, v in re.findall(r"#define\s+(KBHIP_[A-Z_]+)\s+(-?\d+)", src)}
    assert (defs["KBHIP_ALLOCATED"], defs["KBHIP_PIPELINED"], defs["KBHIP_EVICTED"]) == \
        (kbhip.ALLOCATED, kbhip.PIPELINED, kbhip.EVICTED)
    assert (defs["KBHIP_STOP_ALL"], defs["KBHIP_STOP_UNASSIGNED"], defs["KBHIP_STOP_READY"]) == \
        (kbhip.STOP_ALL, kbhip.STOP_UNASSIGNED, kbhip.STOP_READY)


def test_stats_struct_matches_header():
    """kbhip_stats: the ctypes mirror has the header's fields in order."""
    import kbhip
    src = open(os.path.join(ROOT, "include", "kbhip.h")).read()
    body = re.search(r"typedef struct kbhip_stats \{(.*?)\} kbhip_stats;", src, re.S).group(1)
    fields = re.findall(r"\b(double|int64_t)\s+([a-z_0-9]+);", body)
    mirror = list(kbhip.Stats._fields_)
    assert [n for _, n in fields] == [n for n, _ in mirror]
    ctype = {"double": ctypes.c_double, "int64_t": ctypes.c_int64}
    assert all(ctype[t] is m for (t, _), (_, m) in zip(fields, mirror))


def test_host_loop_binary_built():
    """kube-batch-1_amd/_build/kbhost (the C++ host loop over the per-pop ABI)
    is built with the library; without arguments it prints its usage."""
    import subprocess
    exe = os.path.join(ROOT, "kube-batch-1_amd", "_build", "kbhost")
    if not os.path.exists(exe):
        import kbhip
        kbhip.build()
    r = subprocess.run([exe], capture_output=True, text=True, timeout=30)
    assert r.returncode == 2 and "usage" in r.stderr
