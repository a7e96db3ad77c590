"""Generate the constant tables of madrona_basketball_amd/csrc/bb_math.h.

atan(i/8), i = 0..8, as (hi, lo) double pairs, computed with 60-digit
Decimal arithmetic.  Run:  python tools/gen_math_tables.py
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


if __name__ == "__main__":
    main()
