"""Diagnostic: steady-state event timeline of the overlapped pops at C4, full
speed (overlap 1, speculate 2), from the libkbhip_tl.so build (events written
with s_memrealtime, 100 MHz; kbhip_batch.h TL / TLB).  Prints medians of the
gaps between events of pop e and its predecessor — the critical loop.  Never
used for timing claims (the events cost a few stores per pop).

TL events of pop e (one writer each): 0 block 0 started, 4 final merge done,
5 pop e-1's done seen, 6 own candidates published, 7 placement decided,
8 done written, 9 = 1 fast placement / 2 levels, 10 tasks placed, 11 placement
start (after the barrier), 12 wave 1 gathered the list rows, 13 previous
candidates' rows loaded, 14 placement rows read from the row cache, 15 fast /
levels decision known by every wave.
TLB events per block of every 64th pop: 0 start, 1 sorted and 128-merged
(before the previous pop's candidates), 2 saw them, 3 list published, 4 group
list published (mergers).
usage: python profiles/timeline.py [--overlap K] [--out F]"""
import ctypes, json, os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kube-batch-1_amd"))
import kbhip
kbhip.LIB_PATH = os.path.join(ROOT, "kube-batch-1_amd", "_build", "libkbhip_tl.so")
import kbgen
p = "/tmp/kbhip_bench/c4_100000_800000_%d.kbs" % (kbgen.BASE_SEED + 4)
if not os.path.exists(p):
    os.makedirs(os.path.dirname(p), exist_ok=True)
    kbgen.gen_c4(p)
L = kbhip.lib()
L.kbhip_debug_timeline.restype = ctypes.c_int64
L.kbhip_debug_timeline.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int]
SLOTS, EV, SAMPLES, BLOCKS = 32768, 32, 512, 256
W = SLOTS * EV + SAMPLES * BLOCKS * 8
buf = np.zeros(W, dtype=np.uint64)
OVERLAP = int(sys.argv[sys.argv.index("--overlap") + 1]) if "--overlap" in sys.argv else 1
with kbhip.Session(p) as s:
    assert L.kbhip_debug_timeline(s._h, None, 0, 1) == W  # the buffer exists before any kernel runs
    s.set_option("overlap", OVERLAP)
    s.allocate()  # warm
with kbhip.Session(p) as s:
    assert L.kbhip_debug_timeline(s._h, None, 0, 1) == W
    s.set_option("overlap", OVERLAP)
    s.allocate()
    L.kbhip_debug_timeline(s._h, buf.ctypes.data, W, 0)
T = buf[:SLOTS * EV].reshape(SLOTS, EV).astype(np.int64)
B = buf[SLOTS * EV:].reshape(SAMPLES, BLOCKS, 8).astype(np.int64)
valid = (T[:, 0] > 0) & (T[:, 8] > 0) & (T[:, 6] > 0)
idx = np.nonzero(valid)[0]
idx = idx[(idx > 1000) & (idx < 20000)]  # steady state; slots are seq % 32768
idx = idx[valid[idx - 1] & valid[idx - 2]]
cur, prev, prev2 = T[idx], T[idx - 1], T[idx - 2]
us = lambda x: float(np.median(x)) / 100.0  # 100 MHz ticks -> us
out = {
    "overlap": OVERLAP,
    "pops": int(len(idx)),
    "period (touched e-1 -> touched e)": us(cur[:, 6] - prev[:, 6]),
    "period (done e-1 -> done e)": us(cur[:, 8] - prev[:, 8]),
    "kernel start after done(e-2)": us(cur[:, 0] - prev2[:, 8]),
    "touched(e-1) -> final merge done(e)": us(cur[:, 4] - prev[:, 6]),
    "final merge done -> done(e-1) seen": us(cur[:, 5] - cur[:, 4]),
    "done(e-1) written -> seen": us(cur[:, 5] - prev[:, 8]),
    "done(e-1) seen -> previous candidates' rows loaded": us(cur[:, 13] - cur[:, 5]),
    "done(e-1) seen -> touched(e) published (patch)": us(cur[:, 6] - cur[:, 5]),
    "final merge done -> list rows gathered (wave 1)": us(cur[:, 12] - cur[:, 4]),
    "touched(e) -> placement start (barrier)": us(cur[:, 11] - cur[:, 6]),
    "placement start -> rows from the cache": us(cur[:, 14] - cur[:, 11]),
    "rows from the cache -> fast decision known": us(cur[:, 15] - cur[:, 14]),
    "fast decision known -> placement decided": us(cur[:, 7] - cur[:, 15]),
    "placement decided -> done(e)": us(cur[:, 8] - cur[:, 7]),
    "touched(e-1) -> done(e-1)": us(prev[:, 8] - prev[:, 6]),
    "fast placements": float(np.mean(cur[:, 9] == 1)),
    "tasks per pop": float(np.mean(cur[:, 10])),
}
for fl, nm in ((1, "fast"), (2, "levels")):
    m = cur[:, 9] == fl
    if m.any():
        out[f"{nm}: touched(e) -> placement decided"] = float(np.median(cur[m, 7] - cur[m, 6])) / 100
# per-block events of the sampled pops (seq % 64 == 0)
rows = []
for k in range(SAMPLES):
    seq = None
    for q in range(k * 64, SLOTS, SAMPLES * 64):  # the sampled pop whose slot matches, in the steady window
        if 1000 < q < 20000 and valid[q] and valid[q - 1]:
            seq = q
            break
    if seq is None:
        continue
    b = B[k]
    nb = int(np.count_nonzero(b[:, 0]))
    if nb < 8:
        continue
    b = b[:nb]
    t0, tp = T[seq, 0], T[seq - 1, 6]  # block 0 start; the previous pop's candidates published
    st = b[:, 3] > 0  # blocks that published a list (mergers publish a group list, or nothing for block 0)
    rows.append({
        "blocks": nb,
        "first start": (b[:, 0].min() - t0), "last start": (b[:, 0].max() - t0),
        "merged (median block)": np.median(b[:, 1] - t0), "merged (last block)": (b[:, 1].max() - t0),
        "touched(e-1) published": (tp - t0),
        "saw it (median)": np.median(b[:, 2] - t0), "saw it (last)": (b[:, 2].max() - t0),
        "published (last plain block)": (b[st, 3].max() - t0) if st.any() else 0,
        "group lists published (last)": (b[:, 4].max() - t0),
        "final merge done": (T[seq, 4] - t0),
        "sweep+sort+merge per block (median)": np.median(b[:, 1] - b[:, 0]),
    })
if rows:
    out["per block, us after block 0 started (median over sampled pops)"] = {
        k: round(float(np.median([r[k] for r in rows])) / 100.0, 2) for k in rows[0] if k != "blocks"}
    out["sampled pops"] = len(rows)
line = json.dumps(out, indent=1)
print(line)
if "--out" in sys.argv:
    open(sys.argv[sys.argv.index("--out") + 1], "w").write(line + "\n")
