"""Bank-conflict census of decode_stream_kernel<11,4> after the per-exchange layouts of
sub256_fwd (decode_stream.hip); same per-symbol accounting as decode_c3_model.py."""
import sys
sys.path.insert(0, __file__.rsplit("/", 1)[0])
from bank_model import cycles

M, NA, MS, LG, T, E = 2048, 4, 256, 32, 1024, 8
QS = 292
GS = 8 * QS


def rb(t):
    sg = t // LG
    return (sg >> 3) * GS + (sg & 7) * QS


def L1(i):
    a, b = i >> 5, i & 31
    return 33 * a + (b ^ ((b >> 4) << 2))


def L2(i): return i + 2 * (i >> 5) + 4 * (i >> 6)


acc = [0, 0]


def report(name, fn, kind, reps):
    tot = ideal = 0
    for w in range(T // 64):
        for rep in range(reps):
            c, i = cycles([E * fn(w * 64 + l, rep) for l in range(64)], kind)
            tot += c; ideal += i
    acc[0] += tot; acc[1] += ideal
    print("%-24s %s cycles %5d ideal %5d x%.2f" % (name, kind, tot, ideal, tot / ideal))


report("pass0 store", lambda t, q: (t // MS) * GS + t % MS + q * QS, "w64", 8)
report("sub load", lambda t, r: rb(t) + t % LG + 32 * r, "r64", 8)
report("x1 store", lambda t, r: rb(t) + L1(8 * (t % LG) + r), "w64", 8)
report("x1 load", lambda t, r: rb(t) + L1(t % LG + 32 * r), "r64", 8)
report("x2 store", lambda t, r: rb(t) + L2(64 * (t % LG // 8) + t % 8 + 8 * r), "w64", 8)
report("x2 load", lambda t, k: rb(t) + L2(t % LG + 32 * (k // 4) + 64 * (k % 4)), "r64", 8)
report("final store", lambda t, k: rb(t) + t % LG + 32 * (k // 4) + 64 * (k % 4), "w64", 8)
report("apply reads", lambda t, k: ((2 * t + k // 4) & 7) * QS + ((2 * t + k // 4) >> 3) + (k % 4) * GS, "r64", 8)
print("total %d ideal %d conflict fraction %.3f" % (acc[0], acc[1], 1 - acc[1] / acc[0]))
# layouts are injective inside the region
assert len({L1(i) for i in range(256)}) == 256 and max(L1(i) for i in range(256)) < QS
assert len({L2(i) for i in range(256)}) == 256 and max(L2(i) for i in range(256)) < QS
