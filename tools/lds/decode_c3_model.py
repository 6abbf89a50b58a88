"""Bank-conflict census of decode_stream_kernel<11,4> (C3) LDS accesses per symbol (one wave of
each kind), using tools/lds/bank_model.py. Mirrors the kernel's address arithmetic."""
import sys
sys.path.insert(0, __file__.rsplit("/", 1)[0])
from bank_model import cycles

M, NA = 2048, 4
MS, LG = M // 8, M // 64          # 256-point sub-transforms, 32 lanes each
T = NA * M // 8                   # 1024 threads


def pad2(i): return i + (i >> 5) + 4 * (i >> 6)


QS = ((pad2(MS - 1) + 1 + 3) // 8) * 8 + 4
GS = 8 * QS
print("QS", QS, "GS", GS)
E = 8  # bytes per entry


def report(name, addr_fn, kind, reps):
    tot = ideal = 0
    for w in range(T // 64):
        for rep in range(reps):
            a = [addr_fn(w * 64 + l, rep) for l in range(64)]
            c, i = cycles(a, kind)
            tot += c; ideal += i
    print("%-34s %s  cycles %6d  ideal %6d  x%.2f" % (name, kind, tot, ideal, tot / ideal))
    return tot, ideal


def region_base(t0):
    sg = t0 // LG
    return (sg >> 3) * GS + (sg & 7) * QS


acc = [0, 0]
def add(r):
    acc[0] += r[0]; acc[1] += r[1]

# pass 0 store: thread t0 -> n = t0 % MS, g = t0 / MS; e[q*QS] at img + g*GS + pad2(n)
add(report("pass0 store", lambda t, q: E * ((t // MS) * GS + pad2(t % MS) + q * QS), "w64", 8))
# sub-transform initial load: rp = rg + pad2(s); v[r] = rp[pad2(r*LG)]
add(report("sub load (s + 32 r)", lambda t, r: E * (region_base(t) + pad2(t % LG) + pad2(r * LG)), "r64", 8))
# pass-0 store of the sub plan: element 8 s + r
add(report("sub st0 (8 s + r)", lambda t, r: E * (region_base(t) + pad2(8 * (t % LG)) + pad2(r)), "w64", 8))
# pass-1 load: element s + 32 r
add(report("sub ld1 (s + 32 r)", lambda t, r: E * (region_base(t) + pad2(t % LG) + pad2(32 * r)), "r64", 8))
# pass-1 store: o = (s/8)*64 + s%8; element o + 8 r
add(report("sub st1 ((s/8)64 + s%8 + 8r)", lambda t, r: E * (region_base(t) + pad2((t % LG // 8) * 64 + t % 8) + pad2(8 * r)), "w64", 8))
# pass-2 load: u = s + 32 i, element j + 64 r  (i = rep // 4, r = rep % 4)
add(report("sub ld2 (u + 64 r)", lambda t, k: E * (region_base(t) + pad2(t % LG + 32 * (k // 4)) + pad2(64 * (k % 4))), "r64", 8))
# final store: u = s + 32 i, element u + 64 r
add(report("sub st2 (u + 64 r)", lambda t, k: E * (region_base(t) + pad2(t % LG + 32 * (k // 4)) + pad2(64 * (k % 4))), "w64", 8))
# apply reads (KADJ): kk = 2 tid + q; img + (kk & 7) QS + pad2(kk >> 3) + r GS
add(report("apply X reads", lambda t, k: E * (((2 * t + k // 4) & 7) * QS + pad2((2 * t + k // 4) >> 3) + (k % 4) * GS), "r64", 8))
# staging reads: stg + (t/W8) RS + odd + t%W8 + r W8 (odd = 0 here)
W8, RS = M // 8, M + 2
add(report("staging reads", lambda t, r: E * (GS * NA + (t // W8) * RS + t % W8 + r * W8), "r64", 8))
print("total cycles %d ideal %d -> conflict fraction %.3f" % (acc[0], acc[1], 1 - acc[1] / acc[0]))
