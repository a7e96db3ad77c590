"""Generate the constant tables of madrona_basketball_amd/csrc/bb_math.h.

atan(i/8), i = 0..8, as (hi, lo) double pairs, and the Taylor coefficients
of erf at the centres of [0.75 + k/4, 1 + k/4), k = 0..12, computed with
60-digit Decimal arithmetic.  Run:  python tools/gen_math_tables.py
"""
from decimal import Decimal, getcontext

getcontext().prec = 60


def atan_small(x: Decimal) -> Decimal:
    # Taylor series; converges fast for |x| <= 1/8 after halving.
    s, term, n = Decimal(0), x, 0
    x2 = x * x
    while True:
        t = term / (2 * n + 1)
        if abs(t) < Decimal(10) ** -58:
            break
        s += t if n % 2 == 0 else -t
        term *= x2
        n += 1
    return s


def atan_dec(x: Decimal) -> Decimal:
    # atan(x) = 2 atan(x / (1 + sqrt(1 + x^2))), applied until |x| < 0.05
    k = 0
    while abs(x) > Decimal("0.05"):
        x = x / (1 + (1 + x * x).sqrt())
        k += 1
    return atan_small(x) * (2 ** k)


def hi_lo(d: Decimal):
    hi = float(d)
    lo = float(d - Decimal(hi))
    return hi, lo


def main():
    rows = []
    for i in range(9):
        rows.append(hi_lo(atan_dec(Decimal(i) / 8)))
    print("// atan(i/8), i = 0..8  (tools/gen_math_tables.py)")
    print("static constexpr double ATAN_HI[9] = {")
    print(",\n".join(f"    {h!r}" for h, _ in rows) + "};")
    print("static constexpr double ATAN_LO[9] = {")
    print(",\n".join(f"    {l!r}" for _, l in rows) + "};")
    pi = atan_dec(Decimal(1)) * 4
    for name, v in (("PI", pi), ("PIO2", pi / 2)):
        h, l = hi_lo(v)
        print(f"static constexpr double {name}_HI = {h!r};")
        print(f"static constexpr double {name}_LO = {l!r};")


def pi_dec() -> Decimal:
    return atan_dec(Decimal(1)) * 4


def exp_dec(x: Decimal) -> Decimal:
    return x.exp()


def erf_dec(x: Decimal) -> Decimal:
    # Maclaurin series at 60 digits (terms peak near 16^16/16! for x <= 4)
    two_over_sqrtpi = 2 / pi_dec().sqrt()
    s, n, z = Decimal(0), 0, x * x
    term = x  # x^(2n+1) / n!
    while True:
        t = term / (2 * n + 1)
        if n > 10 and abs(t) < Decimal(10) ** -70:
            break
        s += t if n % 2 == 0 else -t
        n += 1
        term = term * z / n
    return two_over_sqrtpi * s


ERF_LO, ERF_W, ERF_K = Decimal("0.75"), Decimal("0.25"), 13


def erf_taylor(c: Decimal, deg: int):
    """a_n = erf^(n)(c) / n!: a_0 = erf(c); with g = erf' = 2/sqrt(pi) e^(-x^2),
    g' = -2 x g gives (n+1) b_(n+1) = -2c b_n - 2 b_(n-1) for g's coefficients
    b_n, and a_(n+1) = b_n / (n+1)."""
    b = [2 / pi_dec().sqrt() * exp_dec(-c * c)]
    b.append(-2 * c * b[0])
    while len(b) < deg:
        n = len(b) - 1
        b.append((-2 * c * b[n] - 2 * b[n - 1]) / (n + 1))
    return [erf_dec(c)] + [b[n] / (n + 1) for n in range(deg)]


def erf_table(tol=Decimal(10) ** -19):
    half = ERF_W / 2
    rows, deg = [], 0
    for k in range(ERF_K):
        c = ERF_LO + ERF_W * k + half
        a = erf_taylor(c, 40)
        # smallest degree whose dropped terms stay below tol on |t| <= w/2
        d = len(a) - 1
        while d > 0 and sum(abs(a[n]) * half ** n for n in range(d, len(a))) < tol:
            d -= 1
        deg = max(deg, d + 1)
        rows.append(a)
    return [[float(r[n]) for n in range(deg + 1)] for r in rows], deg


def main_erf():
    rows, deg = erf_table()
    print(f"// erf Taylor coefficients at c_k = 0.875 + k/4 (k = 0..{ERF_K - 1}), degree {deg}")
    print(f"static constexpr int ERF_TK = {ERF_K}, ERF_TD = {deg};")
    print(f"static constexpr double ERF_TAYLOR[{ERF_K}][{deg + 1}] = {{")
    for r in rows:
        print("    {" + ", ".join(repr(v) for v in r) + "},")
    print("};")


if __name__ == "__main__":
    import sys
    if "--erf" in sys.argv:
        main_erf()
    else:
        main()
