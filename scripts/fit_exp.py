"""Fit the fp64 engine's exp polynomial (csrc/tfg_fastmath.hpp exp_impl):
exp(t) = 1 + t (1 + t P(t)) on |t| <= ln2 / 2 (Cody-Waite's reduced range),
P of degree DEG - 2, by a discrete Remez exchange on the relative error, in
mpmath at 40 digits.  Prints the total degree, the fit's error before fp64
rounding, and P's coefficients as C hex literals, highest degree first.

    python scripts/fit_exp.py DEG      (round 5: DEG = 9, 1.6e-14)
"""
import mpmath as mp, sys
mp.mp.dps=40
DEG=int(sys.argv[1])  # total degree; P has degree DEG-2: exp(t) ~ 1 + t (1 + t P(t))
H=mp.log(2)/2*(1+mp.mpf('1e-6'))
def target(t):  # P(t) = ((exp(t)-1)/t - 1)/t
    if abs(t)<mp.mpf('1e-20'): return mp.mpf(1)/2
    return ((mp.exp(t)-1)/t-1)/t
def approx(c,t): return 1+t*(1+t*mp.polyval(c[::-1],t))
def remez(d,iters=15):
    n=d+2; pts=[-H+2*H*(1-mp.cos(mp.pi*k/(n-1)))/2 for k in range(n)]
    grid=[-H+2*H*k/6000 for k in range(6001)]
    for _ in range(iters):
        rows=[];rhs=[]
        for i,t in enumerate(pts):
            w=t*t/mp.exp(t)
            rows.append([t**j for j in range(d+1)]+[(-1)**i/w if w!=0 else 0]); rhs.append(target(t))
        sol=mp.lu_solve(mp.matrix(rows),mp.matrix(rhs)); c=[sol[j] for j in range(d+1)]
        errs=[(approx(c,t)-mp.exp(t))/mp.exp(t) for t in grid]
        ext=[];cur=None
        for t,e in zip(grid,errs):
            if cur is None or mp.sign(e)!=mp.sign(cur[1]): ext.append((t,e)); cur=(t,e)
            elif abs(e)>abs(cur[1]): ext[-1]=(t,e); cur=(t,e)
        ext=sorted(ext,key=lambda x:-abs(x[1]))[:n]; pts=sorted(x[0] for x in ext)
        if len(pts)<n: break
    return c,max(abs(e) for e in errs)
c,e=remez(DEG-2)
print(DEG, mp.nstr(e,3)); print([float(v).hex() for v in c[::-1]])
