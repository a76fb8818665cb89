"""Model of the half-size pair search (halfscalar.h) for the Go-mode tail:
Euclid on (8L, k) to r1 < 2^127, then the shortest pair with odd k2 among
the code's candidates (v1 if odd, else the shorter of v0, v2) and among a wider
set (v0, v1, v2 and their +-1, +-2 combinations). Prints the fraction of
random k whose odd pair exceeds 130 bits (33 windows) for both.

    python tools/hs_tail_model.py
"""
import random
L = 2**252 + 27742317777372353535851937790883648493
N = 8*L
def bl(x): return abs(x).bit_length()
def run(trials=200000, seed=1):
    rnd = random.Random(seed)
    cnt_base = cnt_ext = 0
    hist_b = {}; hist_e = {}
    for _ in range(trials):
        k = rnd.randrange(L)
        r0, r1, t0, t1 = N, k, 0, 1
        while bl(r1) > 127:
            q = r0 // r1
            r0, r1, t0, t1 = r1, r0 - q*r1, t1, t0 - q*t1
        q = r0 // r1
        r2, t2 = r0 - q*r1, t0 - q*t1
        cands = [(r1,t1),(r0,t0),(r2,t2)]
        cost = lambda v: max(bl(v[0]), bl(v[1]))
        base = [v for v in cands if v[1] & 1]
        # code's pick: v1 if odd else min(v0, v2)
        if t1 & 1: b = cost((r1,t1))
        else: b = min(cost((r0,t0)), cost((r2,t2)))
        ext = list(cands)
        for a in (-2,-1,1,2):
            for (x,y),(u,w) in ((cands[0],cands[1]),(cands[1],cands[2]),(cands[0],cands[2])):
                ext.append((x + a*u, y + a*w))
        e = min(cost(v) for v in ext if v[1] & 1 and v[1] != 0)
        hist_b[b] = hist_b.get(b,0)+1; hist_e[e]=hist_e.get(e,0)+1
        cnt_base += b > 130; cnt_ext += e > 130
    print("base >130:", cnt_base/trials, "ext >130:", cnt_ext/trials)
    print("base max", max(hist_b), "ext max", max(hist_e))
    print(sorted(hist_b.items())[-8:]); print(sorted(hist_e.items())[-8:])
run()
