"""Probe: how many rounds a list-scheduling pass would save in each SOP program -- ops pulled
into an earlier round with a free lane when no slot they read is written in between, their destination is
neither read nor written in between, and their product count does not raise the round's largest K.
Prints rounds before / ops moved / rounds after.  Not used by the build."""
import sys
sys.path.insert(0, __import__('os').path.dirname(__import__('os').path.abspath(__file__)))
import gen_sop as G

def rd(o):
    s = set()
    for x, y, _ in o.prods:
        for t in x + y:
            if not isinstance(t.slot, tuple):
                s.add(t.slot)
    for a, _ in o.adds:
        if not isinstance(a, tuple):
            s.add(a)
    return s

def wr(o):
    s = set()
    if o.dst is not None:
        s.add(o.dst)
    if o.load:
        s.add(o.load[0])
    return s

def compact(p, look=12):
    R = p.rounds
    moved = 0
    for r in range(len(R)):
        if not R[r] or any(o.kind != 'sop' for o in R[r]):
            continue
        kmax = max(len(o.prods) for o in R[r])
        for src in range(r + 1, min(len(R), r + 1 + look)):
            if len(R[r]) >= p.team:
                break
            for o in list(R[src]):
                if len(R[r]) >= p.team:
                    break
                if o.kind != 'sop' or len(o.prods) > kmax:
                    continue
                W = set()
                for rr in range(r, src):
                    for q in R[rr]:
                        W |= wr(q)
                if rd(o) & W:
                    continue
                Rd = set()
                for rr in range(r + 1, src):
                    for q in R[rr]:
                        Rd |= rd(q)
                for q in R[src]:
                    if q is not o:
                        Rd |= rd(q)
                if wr(o) & (Rd | W):
                    continue
                R[r].append(o)
                R[src].remove(o)
                moved += 1
    before = len(R)
    R[:] = [x for x in R if x]
    return moved, before, len(R)

progs = G.build()
for p in progs:
    n0 = len(p.rounds)
    m = compact(p)
    p.finalize()
    print(p.name, n0, m, p.stats())
