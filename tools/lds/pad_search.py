"""Search an LDS padding for the decode's wave-local 256-point sub-transforms (StreamPlan<8,1>:
radix 8, 8, 4) that is bank-conflict-free for every access pattern (tools/lds/bank_model.py)."""
import itertools
import sys
sys.path.insert(0, __file__.rsplit("/", 1)[0])
from bank_model import cycles

E = 8


def patterns():
    # (kind, list of per-instruction element-index functions of lane s in [0, 32))
    P = []
    P.append(("r64", [lambda s, r=r: s + 32 * r for r in range(8)]))                      # L0, L1
    P.append(("w64", [lambda s, r=r: 8 * s + r for r in range(8)]))                       # S0
    P.append(("w64", [lambda s, r=r: 64 * (s // 8) + s % 8 + 8 * r for r in range(8)]))   # S1
    P.append(("r64", [lambda s, i=i, r=r: s + 32 * i + 64 * r for i in range(2) for r in range(4)]))  # L2
    P.append(("w64", [lambda s, i=i, r=r: s + 32 * i + 64 * r for i in range(2) for r in range(4)]))  # S2
    P.append(("w64", [lambda s, q=q: s for q in range(1)]))                                # pass-0 store (n contiguous)
    return P


def score(pad):
    tot = ideal = 0
    for kind, fns in patterns():
        for fn in fns:
            # two lane groups of 32: same sub-transform layout, 2 regions (offset irrelevant in a group)
            a = [E * pad(fn(l % 32)) + (E * 4096 if l >= 32 else 0) for l in range(64)]
            c, i = cycles(a, kind)
            tot += c; ideal += i
    return tot, ideal


def injective(pad, n=256):
    v = [pad(i) for i in range(n)]
    return len(set(v)) == n


cands = []
for c3, c4, c5, c6 in itertools.product(range(0, 3), range(0, 3), range(0, 3), range(0, 5)):
    pad = lambda i, c3=c3, c4=c4, c5=c5, c6=c6: i + c3 * (i >> 3) + c4 * (i >> 4) + c5 * (i >> 5) + c6 * (i >> 6)
    if not injective(pad):
        continue
    t, i = score(pad)
    cands.append((t - i, pad(255) + 1, (c3, c4, c5, c6)))
# xor swizzles of the element index within a 32-block by bits above
for sh, msk in itertools.product(range(3, 8), [1, 3, 7, 15, 31]):
    pad = lambda i, sh=sh, msk=msk: (i & ~31) | ((i ^ ((i >> sh) & msk)) & 31)
    if not injective(pad):
        continue
    t, i = score(pad)
    cands.append((t - i, pad(255) + 1, ("xor", sh, msk)))
cands.sort()
for c in cands[:12]:
    print(c)
print("pad2 (current):", score(lambda i: i + (i >> 5) + 4 * (i >> 6)))
