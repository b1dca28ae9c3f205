"""Fit the fp64 engine's arctangent polynomial (csrc/tfg_fastmath.hpp atan_q):
atan(x) = x + x z Q(z), z = x^2, on |x| <= tan(pi/8) (the octant reduction's
range), Q of degree DEG, by a discrete Remez exchange on the relative error of
atan, in mpmath at 40 digits.  Prints the coefficients as C hex literals
(Q's constant term first) and the fit's error before fp64 rounding.

    python scripts/fit_atan.py [DEG]
"""

import sys

import mpmath as mp

mp.mp.dps = 40
DEG = int(sys.argv[1]) if len(sys.argv) > 1 else 9
B = mp.tan(mp.pi / 8) * (1 + mp.mpf("1e-6"))  # a rounded reduced argument may sit an ulp above tan(pi/8)


def q_exact(z):
    x = mp.sqrt(z)
    if z == 0:
        return mp.mpf(-1) / 3
    return (mp.atan(x) - x) / (x * z)


def rel_err(c, z):
    x = mp.sqrt(z)
    approx = x + x * z * mp.polyval(c[::-1], z)
    return (approx - mp.atan(x)) / mp.atan(x) if z > 0 else mp.mpf(0)


def remez(deg, iters=12):
    zmax = B * B
    n = deg + 2
    pts = [zmax * (1 - mp.cos(mp.pi * k / (n - 1))) / 2 for k in range(n)]
    grid = [zmax * k / 4000 for k in range(1, 4001)]
    for _ in range(iters):
        # solve Q(z_i) + (-1)^i E / w(z_i) = q(z_i), with the relative-error weight w = z x / atan(x)
        rows, rhs = [], []
        for i, z in enumerate(pts):
            x = mp.sqrt(z) if z > 0 else mp.mpf("1e-30")
            w = (x * z) / mp.atan(x) if z > 0 else mp.mpf(0)
            rows.append([z ** j for j in range(deg + 1)] + [(-1) ** i / w if w != 0 else 0])
            rhs.append(q_exact(z))
        sol = mp.lu_solve(mp.matrix(rows), mp.matrix(rhs))
        c = [sol[j] for j in range(deg + 1)]
        errs = [rel_err(c, z) for z in grid]
        # new reference: the extremum of each sign run
        ext, cur = [], None
        for z, e in zip(grid, errs):
            if cur is None or mp.sign(e) != mp.sign(cur[1]):
                ext.append((z, e))
                cur = (z, e)
            elif abs(e) > abs(cur[1]):
                ext[-1] = (z, e)
                cur = (z, e)
        ext = sorted(ext, key=lambda t: -abs(t[1]))[:n]
        pts = sorted(t[0] for t in ext)
        if len(pts) < n:
            break
    return c, max(abs(e) for e in errs)


if __name__ == "__main__":
    c, err = remez(DEG)
    print(f"// degree {DEG} in z on |x| <= tan(pi/8): max relative error {mp.nstr(err, 3)} before rounding")
    for v in c:
        print(float(v).hex())
