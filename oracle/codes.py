"""oracle/codes.py -- TEST INFRASTRUCTURE ONLY: LFSR generator polynomials for the checker.

mimo/config.h:70-75 defines one degree-12 polynomial for S0 and two degree-13 polynomials
for the per-stream S1 codes (NUM_STREAMS 2). N > 2 needs more; these are the next
degree-13 polynomials (ascending, odd) whose liquid-style m-sequence has full period 8191,
verified by tests/test_oracle.py::test_msequence_periods.
"""
S0_POLY = 0o10123
S1_POLYS = (0o20033, 0o20047, 0o20065, 0o20123, 0o20145, 0o20157, 0o20213, 0o20215)


def s1_polynomials(n):
    if n > len(S1_POLYS):
        raise ValueError("at most %d streams supported" % len(S1_POLYS))
    return S1_POLYS[:n]
