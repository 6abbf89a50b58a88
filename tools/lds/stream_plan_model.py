"""Bank-conflict census of decode_stream_kernel's Stockham exchanges (StreamPlan<LOG2M, NA>:
st_store / st_load_t in decode_stream.hip) under two layouts: lds_pad for every exchange, and
the per-exchange layouts (exchange after pass 0: x1, i = 32 a + b at 33 a + (b ^ 4 (b >> 4));
after pass 1: x2, i + 2 (i >> 5) + 4 (i >> 6); later ones lds_pad).
usage: stream_plan_model.py LOG2M NA [LANES]  (LANES: threads that share one wave's lane
groups, 64; a wave-local sub-transform plan passes its group size)"""
import sys
sys.path.insert(0, __file__.rsplit("/", 1)[0])
from bank_model import cycles


def plan(LOG2M, NA):
    M = 1 << LOG2M
    T = NA * M // 8
    P8 = (LOG2M - 2) // 3
    TAIL = (LOG2M - 2) % 3
    NP = P8 + (1 if TAIL else 0) + 1
    radix = [8 if p < P8 else (4 if p == NP - 1 else (1 << TAIL)) for p in range(NP)]
    ns = [1]
    for p in range(NP - 1):
        ns.append(ns[-1] * radix[p])
    return M, T, NP, radix, ns


def pad(i): return i + (i >> 5)
def x1(i): return 33 * (i >> 5) + ((i & 31) ^ (((i >> 4) & 1) << 2))
def x2(i): return i + 2 * (i >> 5) + 4 * (i >> 6)


def census(LOG2M, NA, layouts, group=None):
    M, T, NP, radix, ns = plan(LOG2M, NA)
    PB = 1 << 20   # images far apart (antennas' images never share a lane group here)
    E = 8
    acc = [0, 0]
    out = []
    for p in range(NP):
        R, NS, NB = radix[p], ns[p], M // radix[p]
        bt = 8 // R
        for kind in ("r64", "w64"):
            if kind == "r64" and p == 0:
                continue
            # exchange e: stores of pass e then loads of pass e + 1
            L = layouts(p if kind == "w64" else p - 1, NP)
            tot = ideal = 0
            for w in range((T + 63) // 64):
                for i in range(bt):
                    for r in range(R):
                        addrs = []
                        for l in range(64):
                            t = w * 64 + l
                            if group:
                                t = t % group   # wave-local plan: each lane group its own copy
                            if t >= T:
                                addrs.append(None); continue
                            u = t + i * T
                            g, j = u // NB, u % NB
                            if kind == "r64":
                                e = j + r * NB
                            else:
                                e = (j // NS) * NS * R + j % NS + r * NS
                            addrs.append(E * (g * PB + L(e) + (8192 * E if group and w * 64 + l >= group else 0)))
                        c, ii = cycles(addrs, kind)
                        tot += c; ideal += ii
            acc[0] += tot; acc[1] += ideal
            out.append("p%d %s x%.2f" % (p, kind, tot / ideal))
    return 1 - acc[1] / acc[0], out


if __name__ == "__main__":
    LOG2M, NA = int(sys.argv[1]), int(sys.argv[2])
    group = int(sys.argv[3]) if len(sys.argv) > 3 else None
    allpad = lambda e, NP: pad
    per_ex = lambda e, NP: (x1 if e == 0 else (x2 if e == 1 and NP > 3 or e == 1 and NP == 3 else pad)) if e < NP - 1 else pad
    for name, lay in (("lds_pad", allpad), ("per-exchange", per_ex)):
        f, out = census(LOG2M, NA, lay, group)
        print("%-13s conflict fraction %.3f  %s" % (name, f, " ".join(out)))
    M = 1 << LOG2M
    print("footprints: x1 %d x2 %d lds_pad %d" % (max(x1(i) for i in range(M)) + 1,
          max(x2(i) for i in range(M)) + 1, pad(M - 1) + 1))
