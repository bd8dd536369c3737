#!/usr/bin/env python3
"""The Mills-ratio polynomial of hedge_env.hip `mills()`: R(a) = Phi(-a) / phi(a) =
sqrt(pi/2) erfcx(a / sqrt 2) on a in [0, 38.6] as a degree-14 polynomial in
u = A - B / (a + c), c = 5 (a Chebyshev least-squares fit at 4000 Chebyshev nodes in
u, re-expanded in powers of u).  Prints A, B, the coefficients (highest degree first,
for Horner) and the relative error of phi(a) R(a) against scipy.special.ndtr(-a),
evaluated in f64 the way the kernel does."""
import numpy as np
from numpy.polynomial import chebyshev as C
from scipy.special import erfcx, ndtr


def R(x):
    return np.sqrt(np.pi / 2) * erfcx(x / np.sqrt(2))


def main(XM=38.6, c=5.0, deg=14):   # round 3: deg=16 (1.7e-12); before it c=3.5, deg=20
    tm = (XM - c) / (XM + c)
    k = 2 / (tm + 1)
    n = 4000
    u = np.cos(np.pi * (np.arange(n) + 0.5) / n)
    t = (u + 1) / k - 1
    x = c * (1 + t) / (1 - t)
    pc = C.cheb2poly(C.chebfit(u, R(x), deg))
    A, B = 2 * k - 1, 2 * c * k
    print("A %.17g B %.17g" % (A, B))
    print(",\n".join("    %.17g" % v for v in pc[::-1]))
    a = np.linspace(0, 37.4, 400001)
    uu = A - B * (1.0 / (a + c))
    y = np.zeros_like(uu)
    for co in pc[::-1]:
        y = y * uu + co
    Q = np.exp(-0.5 * a * a) / np.sqrt(2 * np.pi) * y
    ok = ndtr(-a) > 0
    print("max relative error of Q: %.3e" % np.max(np.abs(Q[ok] / ndtr(-a)[ok] - 1)))


if __name__ == "__main__":
    main()
