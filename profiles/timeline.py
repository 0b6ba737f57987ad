"""Diagnostic: steady-state event timeline of the overlapped pops at C4, full
speed (overlap 1, speculate 2), from the libkbhip_tl.so build (events written
with s_memrealtime, 100 MHz, by kbhip_batch.h TL / TL_MAX).  Prints the median
gaps between events of pop e and of its predecessor, which show the critical
loop.  Never used for timing claims (the events cost a few stores per pop).

Events per pop e: 0 first block started, 1 last block saw pop e-1's candidates,
2 last block stored its list, 3 last group list stored, 4 final merge done,
5 pop e-1's done seen, 6 own candidates published, 7 placement decided,
8 done written; 9 = 1 fast placement / 2 levels; 10 = tasks placed; 11 placement
start (after the barrier); 12 wave 1 gathered the list rows; 13 previous
candidates' rows loaded (the last lane's store); 14 placement rows read from
the row cache; 15 fast / levels decision known by every wave; 16 / 17 first /
last block start; 18 / 19 last / first block done with its sort and 128-merge.
usage: python profiles/timeline.py [--out F]"""
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
W = 32768 * 32
buf = np.zeros(W, dtype=np.uint64)
with kbhip.Session(p) as s:
    assert L.kbhip_debug_timeline(s._h, None, 0, 1) == W  # the buffer exists before any kernel runs
    s.allocate()  # warm
with kbhip.Session(p) as s:
    assert L.kbhip_debug_timeline(s._h, None, 0, 1) == W
    s.allocate()
    L.kbhip_debug_timeline(s._h, buf.ctypes.data, W, 0)
T = buf.reshape(32768, 32).astype(np.int64)
for ev in (16, 19):  # minima were stored inverted (atomic max of ~t)
    T[:, ev] = np.where(T[:, ev] != 0, ~T[:, ev], 0)
valid = (T[:, 0] > 0) & (T[:, 8] > 0) & (T[:, 6] > 0)
idx = np.nonzero(valid)[0]
# consecutive pops only, skip the first 1000 (ramp) — slots are seq % 32768
idx = idx[(idx > 1000) & (idx < 20000)]
idx = idx[valid[idx - 1]]
cur, prev = T[idx], T[idx - 1]
us = lambda x: float(np.median(x)) / 100.0  # 100 MHz ticks -> us
out = {
    "pops": int(len(idx)),
    "period (touched e-1 -> touched e)": us(cur[:, 6] - prev[:, 6]),
    "period (done e-1 -> done e)": us(cur[:, 8] - prev[:, 8]),
    "kernel start after done(e-2)": us(cur[:, 0] - T[idx - 2, 8]),
    "e start -> last block saw touched(e-1)": us(cur[:, 1] - cur[:, 0]),
    "touched(e-1) published -> last block saw it": us(cur[:, 1] - prev[:, 6]),
    "last block saw touched -> last block list stored": us(cur[:, 2] - cur[:, 1]),
    "last block list -> last group list": us(cur[:, 3] - cur[:, 2]),
    "last group list -> final merge done": us(cur[:, 4] - cur[:, 3]),
    "final merge done -> done(e-1) seen": us(cur[:, 5] - cur[:, 4]),
    "done(e-1) written -> seen": us(cur[:, 5] - prev[:, 8]),
    "done(e-1) seen -> touched(e) published (patch)": us(cur[:, 6] - cur[:, 5]),
    "touched(e) -> placement decided": us(cur[:, 7] - cur[:, 6]),
    "done(e-1) seen -> previous candidates' rows loaded": us(cur[:, 13] - cur[:, 5]),
    "final merge done -> list rows gathered (wave 1)": us(cur[:, 12] - cur[:, 4]),
    "touched(e) -> placement start (barrier)": us(cur[:, 11] - cur[:, 6]),
    "placement start -> placement decided": us(cur[:, 7] - cur[:, 11]),
    "placement start -> rows from the cache": us(cur[:, 14] - cur[:, 11]),
    "rows from the cache -> fast decision known": us(cur[:, 15] - cur[:, 14]),
    "fast decision known -> placement decided": us(cur[:, 7] - cur[:, 15]),
    "placement decided -> done(e)": us(cur[:, 8] - cur[:, 7]),
    "touched(e-1) -> done(e-1)": us(prev[:, 8] - prev[:, 6]),
    "touched(e-1) -> final merge done(e)": us(cur[:, 4] - prev[:, 6]),
    "kernel start -> first block start": us(cur[:, 16] - cur[:, 0]),
    "first block start -> last block start": us(cur[:, 17] - cur[:, 16]),
    "kernel start -> first block merged (before touched)": us(cur[:, 19] - cur[:, 0]),
    "kernel start -> last block merged (before touched)": us(cur[:, 18] - cur[:, 0]),
    "touched(e-1) published -> last block merged (before touched)": us(cur[:, 18] - prev[:, 6]),
    "fast placements": float(np.mean(cur[:, 9] == 1)),
    "tasks per pop": float(np.mean(cur[:, 10])),
}
for fl, nm in ((1, "fast"), (2, "levels")):
    m = cur[:, 9] == fl
    if m.any():
        out[f"{nm}: touched(e) -> placement decided"] = float(np.median(cur[m, 7] - cur[m, 6])) / 100
        out[f"{nm}: tasks"] = float(np.mean(cur[m, 10]))
line = json.dumps(out, indent=1)
print(line)
if "--out" in sys.argv:
    open(sys.argv[sys.argv.index("--out") + 1], "w").write(line + "\n")
