"""Per-exchange LDS layouts for the decode's wave-local 256-point sub-transforms: each exchange
(a write pattern then a read pattern, tools/lds/bank_model.py banking) may use its own additive
padding addr(i) = i + sum_k c_k floor(i / 2^k) (offsets stay compile-time immediates). Lists
the conflict-free ones with the smallest footprint."""
import itertools
import sys
sys.path.insert(0, __file__.rsplit("/", 1)[0])
from bank_model import cycles

E = 8
EXCH = {
    "x0 pass0->sub (n ; s+32r)": (("w64", [lambda s, r=0: s]), ("r64", [lambda s, r=r: s + 32 * r for r in range(8)])),
    "x1 (8s+r ; s+32r)": (("w64", [lambda s, r=r: 8 * s + r for r in range(8)]),
                          ("r64", [lambda s, r=r: s + 32 * r for r in range(8)])),
    "x2 (64(s/8)+s%8+8r ; u+64r)": (("w64", [lambda s, r=r: 64 * (s // 8) + s % 8 + 8 * r for r in range(8)]),
                                    ("r64", [lambda s, i=i, r=r: s + 32 * i + 64 * r for i in range(2) for r in range(4)])),
    "x3 (u+64r ; -)": (("w64", [lambda s, i=i, r=r: s + 32 * i + 64 * r for i in range(2) for r in range(4)]), None),
}


def cost(pad, pats):
    tot = ideal = 0
    for kind, fns in pats:
        for fn in fns:
            a = [E * pad(fn(l % 32)) + (E * 8192 if l >= 32 else 0) for l in range(64)]
            c, i = cycles(a, kind)
            tot += c; ideal += i
    return tot - ideal


for name, (w, r) in EXCH.items():
    pats = [w] + ([r] if r else [])
    res = []
    for cs in itertools.product(range(0, 3), range(0, 3), range(0, 3), range(0, 3), range(0, 5)):
        pad = lambda i, cs=cs: i + sum(c * (i >> k) for c, k in zip(cs, (2, 3, 4, 5, 6)))
        if len({pad(i) for i in range(256)}) != 256:
            continue
        res.append((cost(pad, pats), pad(255) + 1, cs))
    res.sort()
    print(name, res[:4])
