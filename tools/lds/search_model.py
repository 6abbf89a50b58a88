"""Bank-conflict census of search_ls_wave_kernel<13,11> LDS exchanges (one slot pair): the
wave-local 1024-point transforms (RegPlan<10,16>: radix 16, 4, 16) and the block exchange,
with the region's lds_pad layout and with the x1 layout of wave1024 (est_kernels.hip)."""
import sys
sys.path.insert(0, __file__.rsplit("/", 1)[0])
from bank_model import cycles

E = 8


def pad(i): return i + (i >> 5)


def x1(i):
    a, b = i >> 5, i & 31
    return 33 * a + (b ^ (((b >> 4) & 1) << 3))


def run(name, fn, kind, reps, waves=8):
    tot = ideal = 0
    for w in range(waves):
        for r in range(reps):
            c, i = cycles([E * fn(w, l, r) for l in range(64)], kind)
            tot += c; ideal += i
    return tot, ideal


for label, L1 in (("lds_pad", pad), ("x1 layout", x1)):
    acc = [0, 0]
    rows = [
        ("block store", lambda w, l, k: (k // 2) * 1056 + pad(w * 64 + l + 512 * (k % 2)), "w64", 16, 1),
        ("wave load lane+64e", lambda w, l, e: pad(l + 64 * e), "r64", 16, 1),
        ("st0 16l+r", lambda w, l, r: L1(16 * l + r), "w64", 16, 3),
        ("ld1 j+256r", lambda w, l, k: L1(l + 64 * (k // 4) + 256 * (k % 4)), "r64", 16, 3),
        ("st1 o+16r", lambda w, l, k: pad(((l + 64 * (k // 4)) // 16) * 64 + (l + 64 * (k // 4)) % 16 + 16 * (k % 4)), "w64", 16, 3),
        ("ld2 l+64r", lambda w, l, r: pad(l + 64 * r), "r64", 16, 3),
        ("inv store l+64e", lambda w, l, e: pad(l + 64 * e), "w64", 16, 2),
        ("block load", lambda w, l, k: (k // 2) * 1056 + pad(w * 64 + l + 512 * (k % 2)), "r64", 16, 2),
    ]
    for name, fn, kind, reps, mult in rows:
        t, i = run(name, fn, kind, reps)
        acc[0] += t * mult; acc[1] += i * mult
        print("  %-18s %s x%.2f" % (name, kind, t / i))
    print("%s: cycles %d ideal %d conflict fraction %.3f" % (label, acc[0], acc[1], 1 - acc[1] / acc[0]))
assert len({x1(i) for i in range(1024)}) == 1024 and max(x1(i) for i in range(1024)) < 1056
