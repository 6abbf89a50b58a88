"""LDS bank-conflict model of a wave's 8-byte accesses (gfx950 per-instruction lane groups and
bank mapping, /opt/skills/guides/MI355X_MICROARCH.md LDS table): returns the cycles of one wave
instruction and the conflict-free cycles."""
from collections import defaultdict

READ_B64_GROUPS = [list(range(0, 32)), list(range(32, 64))]
WRITE_B64_GROUPS = [list(range(16 * g, 16 * g + 16)) for g in range(4)]


def cycles(addrs, kind):
    """addrs: 64 byte addresses (None = inactive lane) of an 8-byte access"""
    if kind == "r64":
        groups, nb = READ_B64_GROUPS, 64
    else:
        groups, nb = WRITE_B64_GROUPS, 32
    tot = 0
    for g in groups:
        banks = defaultdict(set)
        for l in g:
            a = addrs[l]
            if a is None:
                continue
            for d in (a // 4, a // 4 + 1):
                banks[d % nb].add(d)
        tot += max((len(v) for v in banks.values()), default=0)
    ideal = len(groups)                 # one LDS cycle per lane group when conflict-free
    return tot, ideal
