#!/usr/bin/env python3
"""Generate the SOP ("sum of products") team programs of liblcv.so (csrc/lcv_sop_programs.inc): the
Miller loop (line precompute + accumulation) and the final exponentiation of the two-pairing check
inside FastAggregateVerify (reference call site sync-protocol.md:464).

Why sums of products (round 1's team interpreter ran one Fp multiplication per lane per round):
on gfx950 a fully reduced Montgomery product costs 288 v_mad_u64_u32, and an interpreter that issues
one product per lane per round spends more on operand evaluation, LIN lanes and round latency than on
the product (profiles/r02_v1: VALU busy 0.42-0.50, 1.0-2.4 waves/SIMD).  Here every lane op is

    dst = REDC( sum_k  m_k * X_k * Y_k  +  R * (c_0 v_a + c_1 v_b) )  mod p          (R = 2^384)

with X_k, Y_k = (+-v) (+-v) operand pairs read from the team's LDS slots.  The K products accumulate
unreduced in a 25-word double-width accumulator and ONE Montgomery reduction closes the op (lazy
reduction): an Fp12 squaring is 12 lanes x 7 products in one round, a cyclotomic squaring 12 lanes x 3
products in one round, a sparse line product 12 lanes x 6 products.  Lanes of a team are one Fp
coefficient each (team 12 = one Fp12), five teams per wave.

Programs are explicit lists of rounds written at the Fp-coefficient level from the tower formulas
(Fp12 = Fp2[w]/(w^6 - xi), xi = 1 + u, coefficient order g0..g5 of w^i).  An op may write a slot that
ops of the same round read (in place): the team lives in one wave, every LDS read of a round is issued
before its single store, and LDS operations of one wave complete in order.

The generator EMULATES every program with Python integers exactly as the device computes (Montgomery
representatives, unreduced accumulator, REDC, the header's conditional-subtraction count) and checks
accumulator and result bounds and the results against oracle/bls12_381.py.

    python tools/gen_sop.py [--check] [--out path]
"""
from __future__ import annotations

import argparse
import os
import random
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

P = 0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFAAAB
X_ABS = 0xD201000000010000
R = 1 << 384
RINV = pow(R, -1, P)
NP = (-pow(P, -1, R)) % R          # -p^-1 mod R (REDC)
ACC_BITS = 800                     # 25 x 32-bit accumulator words
L28, M28 = 28, (1 << 28) - 1       # device limbs: 14 x 28 bits per value, 28 64-bit column accumulators
NLIMB = 14
KARATSUBA = True                   # device products: one Karatsuba level where the columns allow
MAXK = 15
SLOT_MASK = 0xFFF
NEG = 0x8000                       # term halfword: slot | NEG
PCONST = 0x8000                    # product-term halfword: 48 * slot, or PCONST | 48 * constant index
SHADOW_NONE = 0x3FF                # record word 1: no shadow slot


def mont(x):
    return x * R % P


def unmont(x):
    return x * RINV % P


def limb_bounds(v, n=15):
    """Per-limb bounds of a normalised 28-bit-limb value <= v."""
    return [min(M28, v >> (L28 * i)) for i in range(n)]


TB28 = limb_bounds(P)                                  # a term: a value < p or a shadow p - v in (0, p]
PL28 = [(P >> (L28 * i)) & M28 for i in range(NLIMB)]  # p's limbs


# ============================================================================ program representation
class T:
    """An operand term: slot, negated?  (the device reads p - v for a negated term)."""
    __slots__ = ("slot", "neg")

    def __init__(self, slot, neg=False):
        self.slot, self.neg = slot, neg

    def __invert__(self):
        return T(self.slot, not self.neg)

    def __repr__(self):
        return ("-" if self.neg else "") + f"s{self.slot}"


class Op:
    """dst = REDC(sum m*X*Y + R*sum c*v) (kind 'sop'), or dst = (add-in value)^-1 (kind 'inv')."""

    def __init__(self, dst, prods=(), adds=(), kind="sop", load=None, emit=None):
        self.dst = dst
        # a negative multiplier is folded into X's term signs: m > 0 from here on
        self.prods = [(list(x) if m > 0 else [~t for t in x], list(y), abs(int(m))) for x, y, m in prods]
        # a product with a single constant factor takes the whole sign on the constant (p - c is another
        # constant): the variable's value then needs no shadow slot for this read
        self.prods = [([~t for t in x], [~y[0]], m) if (len(y) == 1 and isinstance(y[0].slot, tuple) and x and
                                                       all(t.neg for t in x)) else (x, y, m)
                      for x, y, m in self.prods]
        self.adds = [(s if isinstance(s, tuple) else int(s), int(c)) for s, c in adds]
        self.kind = kind
        self.load = load    # (ld_slot, io index): side-load of an Fp value from the program's input stream
        self.emit = emit    # io index: the result is also written to the program's output stream
        self.dst_shadow = None   # slot that also receives p - result (Program.apply_shadows)
        self.load_shadow = None  # slot that also receives p - loaded value
        for x, y, m in self.prods:
            assert 1 <= len(x) <= 2 and 1 <= len(y) <= 2 and m != 0
        assert len(self.adds) <= 2


class Program:
    def __init__(self, name, team):
        self.name, self.team = name, team
        self.rounds = []
        self.consts = {}        # value (canonical) -> index
        self.nslots = 0
        self.named = {}         # name -> slot (inputs / outputs the kernel's prologue / epilogue use)
        self.free = []

    # slots
    def alloc(self, name=None):
        if self.free:
            s = self.free.pop()
        else:
            s = self.nslots
            self.nslots += 1
        if name:
            self.named[name] = s
        return s

    def alloc_n(self, n, name=None):
        out = [self.alloc() for _ in range(n)]
        if name:
            for k, s in enumerate(out):
                self.named[f"{name}{k}"] = s
        return out

    def release(self, slots):
        self.free.extend(slots)

    def const(self, v):
        v %= P
        if v not in self.consts:
            self.consts[v] = len(self.consts)
        return ("c", self.consts[v])

    def round(self, ops):
        """Append one round; more ops than lanes are split into consecutive rounds, which is only
        exact when no op of a later part reads a slot an earlier part writes (checked).  A split
        round is cut after sorting its ops by product count (a round costs its largest K on every
        lane), unless that order would read a slot an earlier part wrote; then the given order."""
        ops = [o for o in ops if o is not None]
        assert ops
        dsts = [o.dst for o in ops if o.dst is not None] + [o.load[0] for o in ops if o.load]
        assert len(dsts) == len(set(dsts)), "two ops of a round write one slot"

        def parts(order):
            out, written = [], set()
            for k in range(0, len(order), self.team):
                part = order[k:k + self.team]
                reads = {t.slot for o in part for x, y, _ in o.prods for t in x + y} | {s_ for o in part for s_, _ in o.adds}
                if reads & written:
                    return None
                written |= {o.dst for o in part}
                out.append(part)
            return out
        split = None
        if len(ops) > self.team:
            split = parts(sorted(ops, key=lambda o: -len(o.prods)))
        if split is None:
            split = parts(ops)
        assert split is not None, f"{self.name}: split round reads a slot an earlier part wrote"
        self.rounds.extend(split)

    # ------------------------------------------------------------ negated shadows
    def apply_shadows(self):
        """Remove every negated product-operand read.  A product term -v (read as p - v) costs each lane
        a 12-word subtraction and select per term in every round with any negation (the header's
        flag is wave-uniform), which measured as ~45% of a K = 4 op (tools/microbench/sopbench.hip).
        Instead, the op that produces v (or the round that side-loads it) also stores p - v in a
        shadow slot, once, and the readers read that slot.  Negated constants become constants
        p - c.  Values the program does not produce (the prologue's inputs) get their shadows from
        one extra first round of add-in ops (dst = R * (-1) * v).  Shadow slots are allocated above
        the program's slots by interval colouring over each shadow's live range (written at the end
        of its round, last read in a later round: a slot whose old shadow is last read in round r
        may take a new shadow written in round r, since a round's reads precede its stores)."""
        if getattr(self, "_shadowed", False):
            return
        self._shadowed = True
        producer = {}          # slot -> current value id
        need = {}              # value id -> last round (in the final numbering) that reads -v
        reads = []             # (round index, op, kind, k, j, value id) for rewriting
        inputs = []            # value ids of prologue inputs
        for r, ops in enumerate(self.rounds):
            for o in ops:
                for k, (x, y, m) in enumerate(o.prods):
                    for kind, terms in (("x", x), ("y", y)):
                        for j, t in enumerate(terms):
                            if not t.neg:
                                continue
                            if isinstance(t.slot, tuple):  # constant: use the constant p - c
                                terms[j] = T(self.const(P - self.const_list_value(t.slot)))
                                continue
                            vid = producer.get(t.slot)
                            if vid is None:
                                vid = producer[t.slot] = ("input", t.slot)
                                inputs.append(vid)
                            need[vid] = r
                            reads.append((r, o, kind, k, j, vid))
            for lane, o in enumerate(ops):   # the round's stores follow its reads
                producer[o.dst] = ("op", r, lane)
                if o.load:
                    producer[o.load[0]] = ("load", r, lane)
        # prologue inputs: one extra first round (indices of later rounds shift by one)
        shift = 1 if inputs else 0
        starts = {}
        for vid in need:
            starts[vid] = 0 if vid[0] == "input" else vid[1] + shift
        for vid in list(need):
            need[vid] += shift
        # interval colouring: value live (start, end]; slot free for a new value starting at t if the
        # previous value's end <= t
        order = sorted(need, key=lambda v: (starts[v], need[v]))
        slot_end = []          # per shadow slot: the end of its current value
        shadow = {}
        for vid in order:
            st, en = starts[vid], need[vid]
            for k, e in enumerate(slot_end):
                if e <= st:
                    slot_end[k] = en
                    shadow[vid] = self.nslots + k
                    break
            else:
                shadow[vid] = self.nslots + len(slot_end)
                slot_end.append(en)
        self.nshadow = len(slot_end)
        for r, o, kind, k, j, vid in reads:
            x, y, m = o.prods[k]
            (x if kind == "x" else y)[j] = T(shadow[vid])
        for vid, sh in shadow.items():
            if vid[0] == "op":
                self.rounds[vid[1]][vid[2]].dst_shadow = sh
            elif vid[0] == "load":
                self.rounds[vid[1]][vid[2]].load_shadow = sh
        if inputs:
            ops = [Op(shadow[v], [], [(v[1], -1)]) for v in inputs]
            self.rounds[:0] = [ops[i:i + self.team] for i in range(0, len(ops), self.team)]
            assert len(ops) <= self.team, "more prologue inputs to negate than lanes"
        self.nslots += self.nshadow

    def const_list_value(self, c):
        for v, k in self.consts.items():
            if k == c[1]:
                return v
        raise KeyError(c)

    # ------------------------------------------------------------ finalise: slot numbers of constants
    def fold_doublings(self):
        """A multiplier 2 as a doubled operand (t + t) in rounds where 2 is the only multiplier besides 1
        and the doubled side's two-term flag is already on: the round then needs no m-scaling of X (12
        multiply-adds per product on the device, paid by every product of the round) and no new flag.
        Bounds are unchanged (len(y) * P = 2P = m P).  Idempotent (no m = 2 remains to fold)."""
        for ops in self.rounds:
            prods = [pr for o in ops for pr in o.prods]
            if not any(m != 1 for _, _, m in prods) or any(m not in (1, 2) for _, _, m in prods):
                continue
            x2 = any(len(x) == 2 for x, _, _ in prods)
            y2 = any(len(y) == 2 for _, y, _ in prods)
            if not all(m == 1 or (y2 and len(y) == 1) or (x2 and len(x) == 1) for x, y, m in prods):
                continue
            for o in ops:
                new = []
                for x, y, m in o.prods:
                    if m == 2:
                        if y2 and len(y) == 1:
                            y, m = [y[0], y[0]], 1
                        else:
                            x, m = [x[0], x[0]], 1
                    new.append((x, y, m))
                o.prods = new

    def order_products(self):
        """Each lane's products two-term first (the sum is order-free): the round's per-product masks
        (header w3) then mark fewer product indices, and the device skips the second term's LDS loads
        and the 12-word add wherever no lane of the round needs one.  Idempotent."""
        for ops in self.rounds:
            for o in ops:
                o.prods = sorted(o.prods, key=lambda t: (-(len(t[0]) + len(t[1])), -len(t[0])))

    def finalize(self):
        self.apply_shadows()
        self.fold_doublings()
        self.order_products()
        if 0 not in self.consts:
            self.consts[0] = len(self.consts)
        self.base_const = self.nslots
        self.zero = self.base_const + self.consts[0]
        assert self.base_const + len(self.consts) < SLOT_MASK

    def relabel(self, perm):
        """Renumber the program's slots (perm: old slot -> new slot, a permutation of range(nslots)),
        after finalize: every op's destination / shadow / side-load slot, add-in and product terms and the
        named slots move together, so the program computes the same values (tools/bank_model.py picks
        perm to lower the modelled LDS bank conflicts)."""
        assert sorted(perm) == list(range(self.nslots))

        def m(s):
            return perm[s] if isinstance(s, int) and 0 <= s < self.nslots else s
        for ops in self.rounds:
            for o in ops:
                o.dst = None if o.dst is None else m(o.dst)
                o.dst_shadow = None if o.dst_shadow is None else m(o.dst_shadow)
                o.load_shadow = None if o.load_shadow is None else m(o.load_shadow)
                if o.load:
                    o.load = (m(o.load[0]), o.load[1])
                o.adds = [(m(a), c) for a, c in o.adds]
                for x, y, _ in o.prods:  # new term objects: one T may sit in several places
                    x[:] = [T(m(t.slot), t.neg) for t in x]
                    y[:] = [T(m(t.slot), t.neg) for t in y]
        self.named = {k: m(v) for k, v in self.named.items()}

    def pterm(self, s):
        """Product-term halfword of slot or constant s: PCONST (constant) | the value's byte offset in its
        LDS table; the device address is lds + offset + (flag ? constants - lds : 0) (lcv_sop.hpp
        sop_pterm: four instructions, no compare)."""
        s = self.sl(s)
        h = PCONST | 48 * (s - self.base_const) if s >= self.base_const else 48 * s
        assert 48 * max(self.nslots, len(self.consts)) < PCONST
        return h

    def sl(self, s):
        if isinstance(s, tuple):
            return self.base_const + s[1]
        return s

    def const_list(self):
        out = [0] * len(self.consts)
        for v, k in self.consts.items():
            out[k] = v
        return out

    # ------------------------------------------------------------ bounds: conditional-subtraction steps
    @staticmethod
    def op_bounds(op):
        """(T bound, REDC result bound) with every stored value < p and each term <= p."""
        tmax = 0
        for x, y, m in op.prods:
            tmax += abs(m) * len(x) * P * len(y) * P
        tmax += R * sum(abs(c) for _, c in op.adds) * P
        return tmax, tmax // R + P

    def red_steps(self, op):
        tmax, res = self.op_bounds(op)
        assert tmax < (1 << ACC_BITS), "accumulator overflow"
        k = 0
        while (P << k) <= res:
            k += 1
        return k

    # ------------------------------------------------------------ device column bounds (28-bit limbs)
    @staticmethod
    def col_bound(op, x15):
        """Largest 64-bit column accumulator of `op` on the device (csrc/lcv_sop.hpp sop_exec): every
        operand (a sum of terms, scaled by m) enters the products as normalised 28-bit limbs, so column c
        receives x_i y_j < 2^56 per limb pair, plus the Montgomery reduction's quotient digits times p's
        limbs and the carries."""
        cols = [0] * 28
        for x, y, m in op.prods:
            assert m * len(x) * P < 1 << (420 if x15 else 392)
            bx, by = limb_bounds(m * len(x) * P), limb_bounds(len(y) * P)
            for i in range(15):
                for j in range(14):
                    cols[i + j] += bx[i] * by[j]
        for i in range(14):
            qb = M28 if i < 13 else (1 << 20) - 1
            for j in range(14):
                cols[i + j] += qb * PL28[j]
        return max(cols) + (1 << 40)

    @staticmethod
    def kara_bound(op):
        """Largest |column| of the subtractive Karatsuba middle product D = sum_k (X0 - X1)(Y1 - Y0)
        over the op's products (7-limb halves, signed 64-bit columns on the device; the P0 and P2
        columns are below the schoolbook columns)."""
        cols = [0] * 13
        for x, y, m in op.prods:
            bx, by = limb_bounds(m * len(x) * P), limb_bounds(len(y) * P)
            dx = [max(bx[i], bx[i + 7]) for i in range(7)]
            dy = [max(by[j], by[j + 7]) for j in range(7)]
            for i in range(7):
                for j in range(7):
                    cols[i + j] += dx[i] * dy[j]
        return max(cols) + (1 << 40)

    def round_flags(self, ops):
        """(x15, kara) of a round, checked against the column bounds: x15 when some m X >= 2^392 (X takes
        15 limbs, schoolbook products); otherwise one Karatsuba level when its middle columns fit."""
        x15 = int(any(m * len(x) * P >= 1 << 392 for o in ops for x, _, m in o.prods))
        assert all(self.col_bound(o, x15) < 1 << 64 for o in ops), f"{self.name}: a column exceeds 2^64"
        kara = int(not x15 and KARATSUBA and all(self.kara_bound(o) < 1 << 63 for o in ops))
        return x15, kara

    # ------------------------------------------------------------ encoding
    def encode(self):
        """hdr: 4 u32 per round (wave-uniform):
             w0 = K | nadd << 4 | mflag << 6 | x2 << 7 | y2 << 8 | neg << 9 | inv << 10 | load << 11 |
                  emit << 12 | shadow << 13 | red << 16 | x15 << 21 | kara << 22 | used << 24
                  (x15: some m X >= 2^392; kara: one Karatsuba level in the products)
             w1 = record offset (u32 words), w2 = record words per lane,
             w3 = xmask | ymask << 16: bit k set when some lane's product k has a two-term X (Y); each
                  lane's products are ordered two-term first (Program.order_products), so the device
                  loads and adds a second term only for the product indices that need one
           rec: per lane (T lanes per round; lanes >= used: dst = SLOT_NONE):
             r0 = dst | flags << 12 (1 inv, 2 load, 4 emit) | ld_slot << 16;
             r1 = io index | dst_shadow << 12 | load_shadow << 22  (shadow slots 10 bits, 0x3FF = none);
             r2, r3 = add-in term: slot | coef << 16 (signed 16-bit);  then per product k:
             [x0 | x1 << 16], [y0 | y1 << 16], [m]    (term = slot | NEG; padding = zero const)"""
        self.finalize()
        hdr, rec = [], []
        z = self.zero
        zp = self.pterm(z)
        for ops in self.rounds:
            K = max(len(o.prods) for o in ops)
            assert K <= MAXK
            nadd = max(len(o.adds) for o in ops)
            mflag = any(abs(m) != 1 for o in ops for _, _, m in o.prods)
            x15, kara = self.round_flags(ops)
            x2 = any(len(x) == 2 for o in ops for x, _, _ in o.prods)
            y2 = any(len(y) == 2 for o in ops for _, y, _ in o.prods)
            neg = any(t.neg for o in ops for x, y, _ in o.prods for t in x + y)
            assert not neg, "a negated product term survived apply_shadows (the device has no run-time path)"
            inv = any(o.kind == "inv" for o in ops)
            load = any(o.load for o in ops)
            emit = any(o.emit is not None for o in ops)
            shadow = any(o.dst_shadow is not None or o.load_shadow is not None for o in ops)
            red = max(self.red_steps(o) for o in ops)
            assert red <= 10, "result above 2^392"
            xmask = ymask = 0
            for o in ops:
                for k, (x, y, _) in enumerate(o.prods):
                    xmask |= (len(x) == 2) << k
                    ymask |= (len(y) == 2) << k
            words = 4 + 3 * K
            hdr += [K | nadd << 4 | int(mflag) << 6 | int(x2) << 7 | int(y2) << 8 | int(neg) << 9 | int(inv) << 10 |
                    int(load) << 11 | int(emit) << 12 | int(shadow) << 13 | red << 16 |
                    x15 << 21 | kara << 22 | len(ops) << 24,
                    len(rec), words, xmask | ymask << 16]
            for lane in range(self.team):
                w = [0] * words
                if lane >= len(ops):
                    w[0] = SLOT_MASK
                    w[2] = w[3] = z
                    for k in range(K):
                        w[4 + 3 * k:7 + 3 * k] = [zp | zp << 16, zp | zp << 16, 1]
                    rec += w
                    continue
                o = ops[lane]
                flags = (1 if o.kind == "inv" else 0) | (2 if o.load else 0) | (4 if o.emit is not None else 0)
                # dst None: an emit-only op (its value leaves through the output stream, no slot)
                dst_enc = SLOT_MASK if o.dst is None else self.sl(o.dst)
                w[0] = dst_enc | flags << 12 | ((self.sl(o.load[0]) if o.load else 0) << 16)
                io = (o.load[1] if o.load else o.emit if o.emit is not None else 0)
                assert 0 <= io < 4096
                ds = SHADOW_NONE if o.dst_shadow is None else o.dst_shadow
                ls = SHADOW_NONE if o.load_shadow is None else o.load_shadow
                assert ds <= SHADOW_NONE and ls <= SHADOW_NONE
                w[1] = io | ds << 12 | ls << 22
                assert not (o.load and o.emit is not None)
                for j in range(2):
                    if j < len(o.adds):
                        s, c = o.adds[j]
                        assert -32768 <= c <= 32767
                        w[2 + j] = self.sl(s) | ((c & 0xFFFF) << 16)
                    else:
                        w[2 + j] = z
                for k in range(K):
                    if k < len(o.prods):
                        x, y, m = o.prods[k]
                        if m < 0:
                            x, m = [~t for t in x], -m
                        assert not any(t.neg for t in x + y)
                        xs = [self.pterm(t.slot) for t in x] + [zp] * (2 - len(x))
                        ys = [self.pterm(t.slot) for t in y] + [zp] * (2 - len(y))
                        w[4 + 3 * k:7 + 3 * k] = [xs[0] | xs[1] << 16, ys[0] | ys[1] << 16, m]
                    else:
                        w[4 + 3 * k:7 + 3 * k] = [zp | zp << 16, zp | zp << 16, 1]
                rec += w
        return hdr, rec

    # ------------------------------------------------------------ emulation (device semantics)
    def emulate(self, mem, io_in=None, io_out=None):
        """mem: slot -> Montgomery representative (< p).  Executes the ENCODED program."""
        hdr, rec = self.encode()
        cl = self.const_list()
        for k, v in enumerate(cl):
            mem[self.base_const + k] = mont(v)
        z = self.zero
        for r in range(len(hdr) // 4):
            w0, off, words, w3 = hdr[4 * r], hdr[4 * r + 1], hdr[4 * r + 2], hdr[4 * r + 3]
            K, nadd, mflag, red, used = w0 & 15, (w0 >> 4) & 3, (w0 >> 6) & 1, (w0 >> 16) & 31, w0 >> 24
            writes = []
            for lane in range(self.team):
                w = rec[off + lane * words:off + (lane + 1) * words]
                dst = w[0] & SLOT_MASK
                if lane >= used:
                    assert dst == SLOT_MASK
                    continue

                def term(h):
                    s = (self.base_const if h & PCONST else 0) + (h & (PCONST - 1)) // 48
                    v = mem[s]
                    assert 0 <= v <= P   # a shadow slot holds p - v in (0, p]
                    return v
                acc = 0
                for k in range(K):
                    a, b, m = w[4 + 3 * k:7 + 3 * k]
                    tx, ty = (w3 >> k) & 1, (w3 >> (16 + k)) & 1   # second term loaded at all?
                    zp = self.pterm(z)
                    assert tx or a >> 16 == zp, "a two-term X outside the round's x mask"
                    assert ty or b >> 16 == zp, "a two-term Y outside the round's y mask"
                    X = term(a & 0xFFFF) + (term(a >> 16) if tx else 0)
                    Y = term(b & 0xFFFF) + (term(b >> 16) if ty else 0)
                    if mflag:
                        X *= m
                    else:
                        assert m == 1
                    assert X < (1 << (420 if (w0 >> 21) & 1 else 392)) and Y < (1 << 392)
                    acc += X * Y
                for j in range(nadd):
                    s, c = w[2 + j] & SLOT_MASK, w[2 + j] >> 16
                    c = c - 65536 if c >= 32768 else c
                    v = mem[s]
                    assert 0 <= v <= P
                    acc += R * (abs(c) * ((P - v) if c < 0 else v))
                assert acc < (1 << ACC_BITS)
                m_ = (acc % R) * NP % R
                res = (acc + m_ * P) // R
                for s_ in range(red - 1, -1, -1):
                    if res >= (P << s_):
                        res -= P << s_
                assert res < P, (self.name, r, lane)
                flags = (w[0] >> 12) & 7
                io, dsh, lsh = w[1] & 0xFFF, (w[1] >> 12) & SHADOW_NONE, (w[1] >> 22) & SHADOW_NONE
                shadow = (w0 >> 13) & 1
                if flags & 1:  # inversion of the add-in value (its first term)
                    res = mont(pow(unmont(res), P - 2, P)) if res else 0
                if flags & 2:
                    writes.append(((w[0] >> 16) & SLOT_MASK, io_in[io]))
                    if shadow and lsh != SHADOW_NONE:
                        writes.append((lsh, P - io_in[io]))
                if flags & 4:
                    io_out[io] = res
                if dst != SLOT_MASK:
                    writes.append((dst, res))
                if shadow and dsh != SHADOW_NONE:
                    writes.append((dsh, P - res))
            for s, v in writes:
                mem[s] = v
        return mem

    def stats(self):
        ops = sum(len(r) for r in self.rounds)
        prods = sum(len(o.prods) for r in self.rounds for o in r)
        slots = sum(self.team * max(len(o.prods) for o in r) for r in self.rounds)
        return (f"{self.name}: team {self.team}, {len(self.rounds)} rounds, {ops} ops, {prods} products "
                f"(+{ops} REDC), {100.0 * prods / max(1, slots):.1f}% of product slots used, "
                f"{self.nslots} LDS slots ({self.nslots * 48} B/item), {len(self.consts)} constants")


# ============================================================================ formula helpers
def fp2_prod(x, y, comp, xi=False, m=1, negx=False):
    """Products of component `comp` of (xi *) x*y for Fp2 views x = (x0, x1), y = (y0, y1).
    negx: the xi forms read negated terms of x only, (x0 - x1) y0 - (x0 + x1) y1 and
    (x0 + x1) y0 + (x0 - x1) y1 (so only x's values need shadow slots: Program.apply_shadows)."""
    x0, x1 = x
    y0, y1 = y
    if not xi:
        return [([x0], [y0], m), ([~x1], [y1], m)] if comp == 0 else [([x0], [y1], m), ([x1], [y0], m)]
    if negx:
        if comp == 0:
            return [([x0, ~x1], [y0], m), ([~x0, ~x1], [y1], m)]
        return [([x0, x1], [y0], m), ([x0, ~x1], [y1], m)]
    if comp == 0:   # x0 (y0 - y1) - x1 (y0 + y1)
        return [([x0], [y0, ~y1], m), ([~x1], [y0, y1], m)]
    return [([x0], [y0, y1], m), ([x1], [y0, ~y1], m)]


def fp2_sqr(x, comp, xi=False, m=1):
    """(xi *) x^2: x^2 = (x0 + x1)(x0 - x1) + 2 x0 x1 u."""
    x0, x1 = x
    base = ([x0, x1], [x0, ~x1], m)
    if not xi:
        return [base] if comp == 0 else [([x0], [x1], 2 * m)]
    if comp == 0:
        return [base, ([~x0], [x1], 2 * m)]
    return [base, ([x0], [x1], 2 * m)]


def neg2(x):
    return (~x[0], ~x[1])


def slots2(p, name=None):
    a = p.alloc(name + "0" if name else None)
    b = p.alloc(name + "1" if name else None)
    return (T(a), T(b))


def fp12_slots(p, name=None):
    return [slots2(p, f"{name}{i}_" if name else None) for i in range(6)]


def conj12(f):
    return [g if i % 2 == 0 else neg2(g) for i, g in enumerate(f)]


def dst_of(view):
    assert not view.neg
    return view.slot


def fp12_sqr_ops(f, out):
    """out = f^2 (schoolbook over Fp2, symmetric pairs): 12 ops, <= 7 products each."""
    ops = []
    for k in range(6):
        for comp in range(2):
            prods = []
            for i in range(6):
                for j in range(i, 6):
                    s = i + j
                    if s % 6 != k:
                        continue
                    xi = s >= 6
                    if i == j:
                        prods += fp2_sqr(f[i], comp, xi)
                    else:
                        prods += fp2_prod(f[i], f[j], comp, xi, 2)
            ops.append(Op(dst_of(out[k][comp]), prods))
    return ops


def fp12_mul_ops(a, b, out, negx=False, conj_out=False):
    """out = a*b (dense, schoolbook over Fp2): 12 ops, 12 products each.  negx: negated reads of a only
    (a single-term y read negated through a view moves its sign to x); conj_out: out = conj(a*b) (the
    odd coefficients' products negated, on x)."""
    ops = []
    for k in range(6):
        for comp in range(2):
            prods = []
            for i in range(6):
                j = (k - i) % 6
                prods += fp2_prod(a[i], b[j], comp, xi=(i + j >= 6), negx=negx)
            if conj_out and k % 2:
                prods = [(x, y, -m) for x, y, m in prods]
            if negx:
                prods = [(x if not (len(y) == 1 and y[0].neg) else [~t for t in x], [~y[0]] if len(y) == 1 and y[0].neg else y, m)
                         for x, y, m in prods]
            ops.append(Op(dst_of(out[k][comp]), prods))
    return ops


def fp12_mul_line_ops(f, line, out):
    """out = f * (a + b w^2 + c w^3): 12 ops, 6 products each."""
    a, b, c = line
    ops = []
    for k in range(6):
        for comp in range(2):
            prods = []
            for j, l in ((0, a), (2, b), (3, c)):
                i = (k - j) % 6
                prods += fp2_prod(f[i], l, comp, xi=(i + j >= 6))
            ops.append(Op(dst_of(out[k][comp]), prods))
    return ops


def cyclo_sqr_ops(g, out, cin=1, cout=1):
    """Granger-Scott cyclotomic squaring, one round: z = [3A0 - 2g0, 3 xi C1 + 2g1, 3B0 - 2g2,
    3A1 + 2g3, 3C0 - 2g4, 3B1 + 2g5] with (A0, A1) = (g0^2 + xi g3^2, 2 g0 g3), (B0, B1) from (g1, g4),
    (C0, C1) from (g2, g5).  12 ops, <= 3 products + one add-in each.
    Scaled values (fexp_program's scaled chain): the slots of g hold cin * g and out receives cout * z, so
    the products take m = 3 cout / cin^2 (6 cout / cin^2 for the 2 x y terms) and the add-ins 2 cout / cin:
    (1, 1) m = 3 / 6 (every product of the round m-scaled on the device), (3, 3) m = 1 / 2 (the 2 folds
    into a doubled operand: no m-scaling), (1, 3) m = 9 / 18, add-ins 6."""
    from fractions import Fraction as Fr
    ms, mp_, ma = Fr(3 * cout, cin * cin), Fr(6 * cout, cin * cin), Fr(2 * cout, cin)
    assert ms.denominator == mp_.denominator == ma.denominator == 1, (cin, cout)
    ms, mp_, ma = int(ms), int(mp_), int(ma)
    ops = []
    pairs = {0: (0, 3), 2: (1, 4), 4: (2, 5)}   # output index -> (x0, x1) of its Fp4 square, "0" part
    for k in range(6):
        for comp in range(2):
            add_c = ma if k % 2 else -ma
            gk = g[k][comp]
            adds = [(gk.slot, add_c if not gk.neg else -add_c)]
            if k in (0, 2, 4):   # 3 (x0^2 + xi x1^2) - 2 g_k  with (x0, x1) = (g0, g3) | (g1, g4) | (g2, g5)
                x0, x1 = pairs[k]
                prods = fp2_sqr(g[x0], comp, False, ms) + fp2_sqr(g[x1], comp, True, ms)
            elif k == 3:         # 3 * 2 g0 g3 + 2 g3
                prods = fp2_prod(g[0], g[3], comp, False, mp_)
            elif k == 5:         # 3 * 2 g1 g4 + 2 g5
                prods = fp2_prod(g[1], g[4], comp, False, mp_)
            else:                # k == 1: 3 xi (2 g2 g5) + 2 g1
                prods = fp2_prod(g[2], g[5], comp, True, mp_)
            ops.append(Op(dst_of(out[k][comp]), prods, adds))
    return ops


def scale_ops(p, src, dst, c):
    """dst = c * src for a constant c (12 ops of one product each; views may carry negations)."""
    cc = T(p.const(c))
    return [Op(dst_of(d), [([s], [cc], 1)]) for s, d in zip(flat12(src), flat12(dst))]


def copy_ops(src, dst):
    """dst = src (views may carry negations): add-in only ops."""
    return [Op(dst_of(d), [], [(s.slot, -1 if s.neg else 1)]) for s, d in zip(src, dst)]


def flat12(f):
    return [t for g in f for t in g]


# ============================================================================ Miller loop: lines
PSI_CX = None
PSI_CY = None


def _psi_consts():
    def inv2(a):
        n = pow((a[0] * a[0] + a[1] * a[1]) % P, P - 2, P)
        return (a[0] * n % P, (-a[1]) * n % P)
    return inv2(_fp2_pow((1, 1), (P - 1) // 3)), inv2(_fp2_pow((1, 1), (P - 1) // 2))


def line_program(team=10, p=None, prefix="", rnd=None, line_op=None):
    """One pairing's T walk over |x| (63 doublings, 5 additions; the projective doubling of
    the projective line doubling scaled by 4, no halvings), emitting per step the sparse line
    (a, b, c) = (c00, c01 * (-xP), c11 * yP), 6 Fp values, io index 6 * step + j.
    Fused use (miller_program): the walk's slots are allocated on the given Program `p` under names
    prefix + ..., its rounds go to rnd(ops, step) (step: the Miller step whose line the round computes; -1
    before the walk, nsteps after it) instead of p.round, line value j of a step is the op
    line_op(step, j, prods, adds) instead of an emit, and no slot is released (the walks' rounds are
    interleaved with other rounds afterwards)."""
    fused = p is not None
    if p is None:
        p = Program("lines", team)
    if rnd is None:
        rnd = lambda ops, st: p.round(ops)  # noqa: E731
    if line_op is None:
        line_op = lambda st, j, prods, adds: Op(None, prods, adds, emit=6 * st + j)  # noqa: E731
    qx, qy = slots2(p, prefix + "qx"), slots2(p, prefix + "qy")
    nxP, yP = T(p.alloc(prefix + "nxp")), T(p.alloc(prefix + "yp"))
    X, Y, Z = slots2(p, prefix + "tx"), slots2(p, prefix + "ty"), slots2(p, prefix + "tz")
    B, Cp, J, XY, YZ = (slots2(p) for _ in range(5))
    BmF, BpF = slots2(p), slots2(p)
    C48 = slots2(p)  # 48 C': carries most of 1728 = 36 * 48, so no scaled operand of the T update needs a 15th limb
    # the line values (a, b, c) only leave through the output stream: emit-only ops without LDS slots (r04)
    # the addition step's temporaries reuse the doubling step's (different steps, sequential rounds)
    th, lam, Cc, D, E, F, G = B, Cp, J, XY, YZ, BmF, BpF
    H, GmH = slots2(p), slots2(p)
    one = T(p.const(1))
    # G2 subgroup check of Q (Scott: psi(Q) == [x]Q): psi(Q) = (conj(qx) cx, conj(qy) cy) now; at the end
    # T = [|x|]Q = -[x]Q, so Q is in G2 iff Z != 0, e1 = px Z - X = 0 and e2 = py Z + Y = 0.  The walk's
    # formulas are exact on G2; on a non-member any exceptional case leaves Z = 0 for good (T = Q in an
    # addition gives (0 : 0 : 0), T = -Q gives O, and O stays O), so a non-member is never accepted.
    px, py = slots2(p, prefix + "px"), slots2(p, prefix + "py")
    cx = (T(p.const(PSI_CX[0])), T(p.const(PSI_CX[1])))
    cy = (T(p.const(PSI_CY[0])), T(p.const(PSI_CY[1])))
    rnd([Op(dst_of(px[c]), fp2_prod((qx[0], ~qx[1]), cx, c)) for c in range(2)] +
        [Op(dst_of(py[c]), fp2_prod((qy[0], ~qy[1]), cy, c)) for c in range(2)], -1)
    step = 0

    for bit in bin(X_ABS)[3:]:
        # ---- doubling
        rnd([Op(dst_of(B[c]), fp2_sqr(Y, c)) for c in range(2)] +
            [Op(dst_of(Cp[c]), fp2_sqr(Z, c, xi=True)) for c in range(2)] +
            [Op(dst_of(J[c]), fp2_sqr(X, c)) for c in range(2)] +
            [Op(dst_of(XY[c]), fp2_prod(X, Y, c)) for c in range(2)] +
            [Op(dst_of(YZ[c]), fp2_prod(Y, Z, c)) for c in range(2)], step)
        # line: a = B - 12 C', b = 3 J * nxP, c = 2 YZ * yP ;  B -+ 3E with E = 12 C'.  This round holds
        # only the add-in combinations (no products: one REDC of cost); b and c, single products of
        # round-one values, ride in the next round's idle lanes (it has 6 ops of K = 2 on 10 lanes)
        ops = [Op(dst_of(BmF[c]), [], [(B[c].slot, 1), (Cp[c].slot, -36)]) for c in range(2)]
        ops += [Op(dst_of(BpF[c]), [], [(B[c].slot, 1), (Cp[c].slot, 36)]) for c in range(2)]
        ops += [line_op(step, c, [], [(B[c].slot, 1), (Cp[c].slot, -12)]) for c in range(2)]
        ops += [Op(dst_of(C48[c]), [], [(Cp[c].slot, 48)]) for c in range(2)]
        rnd(ops, step)
        # T: X = 2 XY (B - 3E), Y = (B + 3E)^2 - 1728 C'^2, Z = 8 B YZ, with 1728 C'^2 taken as
        # 36 (48 C0 + 48 C1)(C0 - C1) + 72 (48 C0) C1 u: the scaled operands stay below 2^392 (14 limbs,
        # Karatsuba), where m = 1728 / 3456 on C' itself needed a 15th limb and schoolbook products
        ysq = [[([C48[0], C48[1]], [Cp[0], ~Cp[1]], -36)], [([C48[0]], [Cp[1]], -72)]]
        ops = [Op(dst_of(X[c]), fp2_prod(XY, BmF, c, m=2)) for c in range(2)]
        ops += [Op(dst_of(Y[c]), fp2_sqr(BpF, c) + ysq[c]) for c in range(2)]
        ops += [Op(dst_of(Z[c]), fp2_prod(B, YZ, c, m=8)) for c in range(2)]
        ops += [line_op(step, 2 + c, [([J[c]], [nxP], 3)], []) for c in range(2)]
        ops += [line_op(step, 4 + c, [([YZ[c]], [yP], 2)], []) for c in range(2)]
        rnd(ops, step)
        step += 1
        if bit == "1":
            # ---- addition T + Q: theta = Y - qy Z, lam = X - qx Z
            # (Z on the x side: the negated reads fall on the walk's running value, Q needs no shadows)
            ops = [Op(dst_of(th[c]), fp2_prod(Z, qy, c, m=-1), [(Y[c].slot, 1)]) for c in range(2)]
            ops += [Op(dst_of(lam[c]), fp2_prod(Z, qx, c, m=-1), [(X[c].slot, 1)]) for c in range(2)]
            rnd(ops, step)
            # C = theta^2, D = lam^2; line (theta qx - lam qy, theta * nxP, lam * yP)
            ops = [Op(dst_of(Cc[c]), fp2_sqr(th, c)) for c in range(2)]
            ops += [Op(dst_of(D[c]), fp2_sqr(lam, c)) for c in range(2)]
            ops += [line_op(step, c, fp2_prod(th, qx, c) + fp2_prod(lam, qy, c, m=-1), []) for c in range(2)]
            ops += [line_op(step, 2 + c, [([th[c]], [nxP], 1)], []) for c in range(2)]
            ops += [line_op(step, 4 + c, [([lam[c]], [yP], 1)], []) for c in range(2)]
            rnd(ops, step)
            # E = lam D, F = Z C, G = X D
            ops = [Op(dst_of(E[c]), fp2_prod(lam, D, c)) for c in range(2)]
            ops += [Op(dst_of(F[c]), fp2_prod(Z, Cc, c)) for c in range(2)]
            ops += [Op(dst_of(G[c]), fp2_prod(X, D, c)) for c in range(2)]
            rnd(ops, step)
            # H = E + F - 2G ; G - H = 3G - E - F   (third terms as products with the constant 1)
            ops = [Op(dst_of(H[c]), [([G[c]], [one], -2)], [(E[c].slot, 1), (F[c].slot, 1)]) for c in range(2)]
            ops += [Op(dst_of(GmH[c]), [([F[c]], [one], -1)], [(G[c].slot, 3), (E[c].slot, -1)]) for c in range(2)]
            rnd(ops, step)
            # X = lam H, Y = theta (G - H) - Y E, Z = Z E
            ops = [Op(dst_of(X[c]), fp2_prod(lam, H, c)) for c in range(2)]
            ops += [Op(dst_of(Y[c]), fp2_prod(th, GmH, c) + fp2_prod(Y, E, c, m=-1)) for c in range(2)]
            ops += [Op(dst_of(Z[c]), fp2_prod(Z, E, c)) for c in range(2)]
            rnd(ops, step)
            step += 1
    if not fused:
        p.release([v.slot for f2 in (B, Cp, J, XY, YZ, BmF, BpF, C48, H, GmH) for v in f2])
    e1, e2 = slots2(p, prefix + "e1"), slots2(p, prefix + "e2")
    rnd([Op(dst_of(e1[c]), fp2_prod(Z, px, c), [(X[c].slot, -1)]) for c in range(2)] +
        [Op(dst_of(e2[c]), fp2_prod(Z, py, c), [(Y[c].slot, 1)]) for c in range(2)], step)
    p.nsteps = step
    return p


def acc_program(team=12, nsteps=68, p=None, lines_of=None, rnd=None):
    """Accumulate f <- f^2 * L1(step) * L2(step) over the Miller steps (no squaring in the first and
    in the addition steps, which follow their doubling step in the same loop iteration), then f^x = conj.
    Lines stream in from the line programs' outputs: io index (6 * step + j) for pairing 1 and
    (6 * nsteps + 6 * step + j) for pairing 2, side-loaded into L1/L2 slots one round ahead.
    Fused use (miller_program): f on the given Program `p` (named f...), the lines of step s already in
    the slots lines_of(s) (written by the walks' rounds: no side-loads, so the first and the addition
    steps' identity rounds, which only carried the loads, are left out), rounds to rnd(ops, step)."""
    fused = p is not None
    if p is None:
        p = Program("miller_acc", team)
    if rnd is None:
        rnd = lambda ops, st: p.round(ops)  # noqa: E731
    f = fp12_slots(p, "f")
    if not fused:
        L = [[slots2(p) for _ in range(3)] for _ in range(2)]   # two lines: (a, b, c)
        lines_of = lambda s: L  # noqa: E731
    # step kinds in loop order (dbl, then add when the bit is 1)
    kinds = []
    for bit in bin(X_ABS)[3:]:
        kinds.append("dbl")
        if bit == "1":
            kinds.append("add")
    assert len(kinds) == nsteps

    def loads(step):
        if fused:
            return [None] * 12
        ops = []
        for k in range(2):
            for j in range(3):
                for c in range(2):
                    ops.append((L[k][j][c].slot, (6 * nsteps) * k + 6 * step + 2 * j + c))
        return ops

    first = True
    for s, kind in enumerate(kinds):
        ld = loads(s)
        Ls = lines_of(s)
        if first:
            # f = 1 (set by the prologue): load both lines, then f = L1 * L2 via two sparse products
            if not fused:
                rnd([Op(dst_of(f[0][0]), [], [(f[0][0].slot, 1)], load=ld[0])] +
                    [Op(dst_of(f[i // 2][i % 2]), [], [(f[i // 2][i % 2].slot, 1)], load=ld[i]) for i in range(1, 12)], s)
            first = False
        elif kind == "dbl":
            ops = fp12_sqr_ops(f, f)
            for i, o in enumerate(ops):
                o.load = ld[i]
            rnd(ops, s)
        elif not fused:
            # addition step: no squaring; the loads ride on an identity round
            rnd([Op(dst_of(f[i // 2][i % 2]), [], [(f[i // 2][i % 2].slot, 1)], load=ld[i]) for i in range(12)], s)
        rnd(fp12_mul_line_ops(f, Ls[0], f), s)
        rnd(fp12_mul_line_ops(f, Ls[1], f), s)
    # x < 0: f -> conj(f)
    rnd(copy_ops(flat12(conj12(f)), flat12(f)), nsteps)
    return p


def miller_program(team=32):
    """Latency mode's Miller loop as ONE program (the fan engine runs it one update per block): both
    pairings' T walks (line_program, slots m_* for e(PK, H(m)) and s_* for e(-G1, sig), the latter with
    its G2 subgroup check) and the accumulation (acc_program), the accumulation one step behind the walks
    in the same rounds: block s holds the walks' rounds of step s + 1 beside the accumulation's rounds of
    step s, whose lines the walks wrote in block s - 1 into the LDS slots of buffer s mod 2 (no line
    stream).  ~220 rounds instead of the walk's 217 followed by the accumulation's 205.  The emulation
    (check_miller_fused) must equal the separate programs' f and subgroup verdicts."""
    p = Program("miller", team)
    acc_rounds, walk_rounds = {}, [{}, {}]

    def rec(store):
        return lambda ops, st: store.setdefault(st, []).append(ops)
    nst = 68
    Lb = []  # [buffer][pairing][a b c]: allocated after f (slots 0..11, as in the separate accumulation)

    def lines_of(s):
        if not Lb:
            Lb.extend([[[slots2(p) for _ in range(3)] for _ in range(2)] for _ in range(2)])
        return Lb[s % 2]
    acc_program(nsteps=nst, p=p, lines_of=lines_of, rnd=rec(acc_rounds))

    def line_op(k):
        return lambda st, j, prods, adds: Op(dst_of(Lb[st % 2][k][j // 2][j % 2]), prods, adds)
    for k, prefix in ((0, "m_"), (1, "s_")):
        lp = line_program(p=p, prefix=prefix, rnd=rec(walk_rounds[k]), line_op=line_op(k))
        assert lp.nsteps == nst
    p.nsteps = nst

    def zipped(*seqs):
        for i in range(max(len(q) for q in seqs)):
            ops = []
            for q in seqs:
                if i < len(q):
                    ops += q[i]
            p.round(ops)
    zipped(walk_rounds[0][-1] + walk_rounds[0][0], walk_rounds[1][-1] + walk_rounds[1][0])
    for s in range(nst):
        zipped(walk_rounds[0][s + 1], walk_rounds[1][s + 1], acc_rounds.get(s, []))
    zipped(acc_rounds[nst])
    return p


# ============================================================================ final exponentiation
FROB = None


def _fp2_pow(a, e):
    r = (1, 0)
    while e:
        if e & 1:
            r = ((r[0] * a[0] - r[1] * a[1]) % P, (r[0] * a[1] + r[1] * a[0]) % P)
        a = ((a[0] * a[0] - a[1] * a[1]) % P, (2 * a[0] * a[1]) % P)
        e >>= 1
    return r


def frob_consts():
    global FROB
    if FROB is None:
        FROB = {k: [_fp2_pow((1, 1), i * (P ** k - 1) // 6) for i in range(6)] for k in (1, 2)}
    return FROB


def frob_ops(p, a, k, out):
    """out = a^(p^k): out_i = conj^k(a_i) * gamma_{k,i}."""
    g = frob_consts()[k]
    ops = []
    for i in range(6):
        x0, x1 = a[i]
        if k % 2:
            x1 = ~x1
        for comp in range(2):
            if i == 0:
                src = (x0, x1)[comp]
                ops.append(Op(dst_of(out[i][comp]), [], [(src.slot, -1 if src.neg else 1)]))
                continue
            c0, c1 = g[i]
            cv = (T(p.const(c0)), T(p.const(c1)))
            prods = fp2_prod((x0, x1), cv, comp)
            if c1 == 0:
                prods = [pr for pr in prods if pr[1][0].slot != cv[1].slot]
            ops.append(Op(dst_of(out[i][comp]), prods))
    return ops


def fexp_program_r03(team=12):
    """f^((p^12 - 1)/r) * 3 (result e^3): easy part
    (p^6 - 1)(p^2 + 1) with a team-parallel Fp12 inversion, hard part (x-1)^2 (x+p)(x^2+p^2-1) + 3."""
    scaled = FEXP_SCALED if scaled is None else scaled
    p = Program("fexp", team)
    f = fp12_slots(p, "f")
    c0 = [f[0], f[2], f[4]]   # Fp6 halves in the v basis
    c1 = [f[1], f[3], f[5]]
    # ---- t = c0^2 - v c1^2
    t = [slots2(p) for _ in range(3)]
    ops = []
    for comp in range(2):
        a, b = c0, c1
        ops.append(Op(dst_of(t[0][comp]), fp2_sqr(a[0], comp) + fp2_prod(a[1], a[2], comp, True, 2) +
                      fp2_sqr(b[1], comp, True, -1) + fp2_prod(b[0], b[2], comp, True, -2)))
        ops.append(Op(dst_of(t[1][comp]), fp2_prod(a[0], a[1], comp, False, 2) + fp2_sqr(a[2], comp, True) +
                      fp2_sqr(b[0], comp, False, -1) + fp2_prod(b[1], b[2], comp, True, -2)))
        ops.append(Op(dst_of(t[2][comp]), fp2_sqr(a[1], comp) + fp2_prod(a[0], a[2], comp, False, 2) +
                      fp2_prod(b[0], b[1], comp, False, -2) + fp2_sqr(b[2], comp, True, -1)))
    p.round(ops)
    # ---- s = adj(t): s0 = t0^2 - xi t1 t2, s1 = xi t2^2 - t0 t1, s2 = t1^2 - t0 t2
    s = [slots2(p) for _ in range(3)]
    ops = []
    for comp in range(2):
        ops.append(Op(dst_of(s[0][comp]), fp2_sqr(t[0], comp) + fp2_prod(t[1], t[2], comp, True, -1)))
        ops.append(Op(dst_of(s[1][comp]), fp2_sqr(t[2], comp, True) + fp2_prod(t[0], t[1], comp, False, -1)))
        ops.append(Op(dst_of(s[2][comp]), fp2_sqr(t[1], comp) + fp2_prod(t[0], t[2], comp, False, -1)))
    p.round(ops)
    # ---- d = t0 s0 + xi (t2 s1 + t1 s2)
    d = slots2(p)
    p.round([Op(dst_of(d[c]), fp2_prod(t[0], s[0], c) + fp2_prod(t[2], s[1], c, True) +
                fp2_prod(t[1], s[2], c, True)) for c in range(2)])
    # ---- n = d0^2 + d1^2 ; ninv
    n = T(p.alloc())
    p.round([Op(n.slot, [([d[0]], [d[0]], 1), ([d[1]], [d[1]], 1)])])
    ninv = T(p.alloc())
    p.round([Op(ninv.slot, [], [(n.slot, 1)], kind="inv")])
    # ---- dinv = (d0 ninv, -d1 ninv) ; tinv = s * dinv
    dinv = slots2(p)
    p.round([Op(dst_of(dinv[0]), [([d[0]], [ninv], 1)]), Op(dst_of(dinv[1]), [([d[1]], [ninv], -1)])])
    ti = [slots2(p) for _ in range(3)]
    p.round([Op(dst_of(ti[i][c]), fp2_prod(s[i], dinv, c)) for i in range(3) for c in range(2)])
    # ---- finv = (c0 * ti, -c1 * ti)   (Fp6 products)
    fi = fp12_slots(p)
    fi0 = [fi[0], fi[2], fi[4]]
    fi1 = [fi[1], fi[3], fi[5]]
    ops = []
    for half, src, sign in ((fi0, c0, 1), (fi1, c1, -1)):
        for k in range(3):
            for comp in range(2):
                prods = []
                for i in range(3):
                    j = (k - i) % 3
                    prods += fp2_prod(src[i], ti[j], comp, xi=(i + j >= 3), m=sign)
                ops.append(Op(dst_of(half[k][comp]), prods))
    p.round(ops)
    # ---- t1 = conj(f) * finv (in place over finv) ; m = frob2(t1) * t1 (frob2 into f's slots, m in place)
    p.round(fp12_mul_ops(conj12(f), fi, fi))
    t1 = fi
    p.round(frob_ops(p, t1, 2, f))
    p.round(fp12_mul_ops(f, t1, t1))
    m = t1
    for i in range(6):
        for c in range(2):
            p.named[f"m{i}_{c}"] = m[i][c].slot
    dead = flat12(f) + [x for v in t + s + ti for x in v] + list(d) + list(dinv) + [n, ninv]
    p.release([x.slot for x in dead])
    acc = fp12_slots(p)
    tmp = fp12_slots(p)

    def exp_x(a, out):
        """out = a^|x| (a cyclotomic; `out` must differ from a's slots)."""
        firstsq = True
        for bit in bin(X_ABS)[3:]:
            p.round(cyclo_sqr_ops(a if firstsq else out, out))
            firstsq = False
            if bit == "1":
                p.round(fp12_mul_ops(out, a, out))

    # A = conj(exp_x(m) * m)          (A in tmp)
    exp_x(m, acc)
    p.round(fp12_mul_ops(acc, m, tmp))
    A = conj12(tmp)
    # A2 = conj(exp_x(A) * A)         (A2 in a fresh Fp12; A's slots become the next scratch)
    exp_x(A, acc)
    A2s = fp12_slots(p)
    p.round(fp12_mul_ops(acc, A, A2s))
    A2 = conj12(A2s)
    # Bv = conj(exp_x(A2)) * frob1(A2)  (frob1 into tmp, Bv in place over tmp)
    exp_x(A2, acc)
    p.round(frob_ops(p, A2, 1, tmp))
    p.round(fp12_mul_ops(conj12(acc), tmp, tmp))
    Bv = tmp
    # t = exp_x(exp_x(Bv))             (t in A2's slots)
    exp_x(Bv, acc)
    exp_x(acc, A2s)
    # C = t * frob2(Bv) * conj(Bv)     (frob2 into acc, C in place over A2s)
    p.round(frob_ops(p, Bv, 2, acc))
    p.round(fp12_mul_ops(A2s, acc, A2s))
    p.round(fp12_mul_ops(A2s, conj12(Bv), A2s))
    C = A2s
    # r = C * (cyclo_sqr(m) * m)       (r over m's slots)
    p.round(cyclo_sqr_ops(m, acc))
    p.round(fp12_mul_ops(acc, m, acc))
    p.round(fp12_mul_ops(C, acc, m))
    for i in range(6):
        for c in range(2):
            p.named[f"r{i}_{c}"] = m[i][c].slot
    return p


FEXP_SCALED = os.environ.get("LCV_SOP_FEXP_SCALED", "1") == "1"   # A/B: 0 = round 5's m-scaled chains


def fexp_program(team=12, scaled=None):
    """f^((p^12 - 1)/r) * 3 (result e^3), three live Fp12 values in the hard part (r04): easy part
    (p^6 - 1)(p^2 + 1) with a team-parallel Fp12 inversion whose temporaries are released as soon as
    they die, then with m = f^((p^6 - 1)(p^2 + 1)), x < 0, e() = exponentiation by |x| (e(a) = a^-x):
        F2 = m^3 (cyclotomic square times m, once, first)
        A  = conj(e(m) m) = m^(x - 1)                  (into m's slots, conjugated by the products)
        A2 = conj(e(A) A) = m^((x - 1)^2)               (in place)
        Bv = conj(e(A2)) frob1(A2) = A2^(x + p)          (frob1 in place, then the product)
        F2 = F2 frob2(Bv) conj(Bv);  F3 = e(Bv);  F1 = e(F3)
        r  = F1 F2 = Bv^(x^2 + p^2 - 1) m^3              (the r03 order's value, fexp_program_r03)
    Every product reads negated values only on its x side (fp2_prod negx, the exponentiation's running
    value), so the chains' bases need no shadow slots: LDS per item 79 -> fewer slots, a third wave per
    SIMD."""
    scaled = FEXP_SCALED if scaled is None else scaled
    p = Program("fexp", team)
    f = fp12_slots(p, "f")
    c0 = [f[0], f[2], f[4]]   # Fp6 halves in the v basis
    c1 = [f[1], f[3], f[5]]
    rel = lambda vs: p.release([x.slot for v in vs for x in (v if isinstance(v, tuple) else (v,))])  # noqa: E731
    # ---- t = c0^2 - v c1^2
    t = [slots2(p) for _ in range(3)]
    ops = []
    for comp in range(2):
        a, b = c0, c1
        ops.append(Op(dst_of(t[0][comp]), fp2_sqr(a[0], comp) + fp2_prod(a[1], a[2], comp, True, 2) +
                      fp2_sqr(b[1], comp, True, -1) + fp2_prod(b[0], b[2], comp, True, -2)))
        ops.append(Op(dst_of(t[1][comp]), fp2_prod(a[0], a[1], comp, False, 2) + fp2_sqr(a[2], comp, True) +
                      fp2_sqr(b[0], comp, False, -1) + fp2_prod(b[1], b[2], comp, True, -2)))
        ops.append(Op(dst_of(t[2][comp]), fp2_sqr(a[1], comp) + fp2_prod(a[0], a[2], comp, False, 2) +
                      fp2_prod(b[0], b[1], comp, False, -2) + fp2_sqr(b[2], comp, True, -1)))
    p.round(ops)
    # ---- s = adj(t): s0 = t0^2 - xi t1 t2, s1 = xi t2^2 - t0 t1, s2 = t1^2 - t0 t2
    s_ = [slots2(p) for _ in range(3)]
    ops = []
    for comp in range(2):
        ops.append(Op(dst_of(s_[0][comp]), fp2_sqr(t[0], comp) + fp2_prod(t[1], t[2], comp, True, -1)))
        ops.append(Op(dst_of(s_[1][comp]), fp2_sqr(t[2], comp, True) + fp2_prod(t[0], t[1], comp, False, -1)))
        ops.append(Op(dst_of(s_[2][comp]), fp2_sqr(t[1], comp) + fp2_prod(t[0], t[2], comp, False, -1)))
    p.round(ops)
    # ---- d = t0 s0 + xi (t2 s1 + t1 s2)
    d = slots2(p)
    p.round([Op(dst_of(d[c]), fp2_prod(t[0], s_[0], c) + fp2_prod(t[2], s_[1], c, True) +
                fp2_prod(t[1], s_[2], c, True)) for c in range(2)])
    rel(t)
    # ---- n = d0^2 + d1^2 ; ninv
    n = T(p.alloc())
    p.round([Op(n.slot, [([d[0]], [d[0]], 1), ([d[1]], [d[1]], 1)])])
    ninv = T(p.alloc())
    p.round([Op(ninv.slot, [], [(n.slot, 1)], kind="inv")])
    rel([n])
    # ---- dinv = (d0 ninv, -d1 ninv) ; tinv = s * dinv
    dinv = slots2(p)
    p.round([Op(dst_of(dinv[0]), [([d[0]], [ninv], 1)]), Op(dst_of(dinv[1]), [([d[1]], [ninv], -1)])])
    rel([d, ninv])
    ti = [slots2(p) for _ in range(3)]
    p.round([Op(dst_of(ti[i][c]), fp2_prod(s_[i], dinv, c)) for i in range(3) for c in range(2)])
    rel(s_ + [dinv])
    # ---- finv = (c0 * ti, -c1 * ti)   (Fp6 products)
    fi = fp12_slots(p)
    fi0 = [fi[0], fi[2], fi[4]]
    fi1 = [fi[1], fi[3], fi[5]]
    ops = []
    for half, src, sign in ((fi0, c0, 1), (fi1, c1, -1)):
        for k in range(3):
            for comp in range(2):
                prods = []
                for i in range(3):
                    j = (k - i) % 3
                    prods += fp2_prod(src[i], ti[j], comp, xi=(i + j >= 3), m=sign)
                ops.append(Op(dst_of(half[k][comp]), prods))
    p.round(ops)
    rel(ti)
    # ---- t1 = conj(f) * finv (in place over finv) ; m = frob2(t1) * t1 (frob2 into f's slots, m in place)
    p.round(fp12_mul_ops(conj12(f), fi, fi))
    t1 = fi
    p.round(frob_ops(p, t1, 2, f))
    p.round(fp12_mul_ops(f, t1, t1))
    m = t1
    for i in range(6):
        for c in range(2):
            p.named[f"m{i}_{c}"] = m[i][c].slot
    rel(flat12(f))
    F1 = m
    F2 = fp12_slots(p)
    F3 = fp12_slots(p)

    # Scaled chains (scaled = FEXP_SCALED, r06): each exponentiation's running value is stored as 3 z, so its
    # 62 squarings after the first are Granger-Scott with m = 1 (products) and 2 (folded into a doubled
    # operand): no m-scaled product rounds (the device's m X costs 12 multiply-adds and as many moves per
    # product).  The first squaring reads the unscaled base (m = 9), the multiplications 3 z * a keep the
    # scale (the base a unscaled), and each chain result that becomes a base or the output is brought back
    # by a product with the constant 1/3 (a one-product round): 5 such rounds against 310 unscaled squarings.
    inv3 = pow(3, -1, P)

    def exp_x(a, out):
        """out = a^|x| (a cyclotomic; `out` must differ from a's slots); negated reads on out only.
        scaled: out holds 3 a^|x|."""
        firstsq = True
        for bit in bin(X_ABS)[3:]:
            if scaled:
                p.round(cyclo_sqr_ops(a if firstsq else out, out, 1 if firstsq else 3, 3))
            else:
                p.round(cyclo_sqr_ops(a if firstsq else out, out))
            firstsq = False
            if bit == "1":
                p.round(fp12_mul_ops(out, a, out, negx=True))

    def unscale(v):
        if scaled:
            p.round(scale_ops(p, v, v, inv3))

    # F2 = m^3 (negated reads on m, whose shadows the squarings need anyway)
    p.round(cyclo_sqr_ops(F1, F2))
    p.round(fp12_mul_ops(F1, F2, F2, negx=True))
    # A = conj(e(m) m) into F1
    exp_x(F1, F3)
    p.round(fp12_mul_ops(F3, F1, F1, negx=True, conj_out=True))
    unscale(F1)
    # A2 = conj(e(A) A) into F1
    exp_x(F1, F3)
    p.round(fp12_mul_ops(F3, F1, F1, negx=True, conj_out=True))
    unscale(F1)
    # Bv = conj(e(A2)) frob1(A2) into F1
    exp_x(F1, F3)
    p.round(frob_ops(p, F1, 1, F1))
    p.round(fp12_mul_ops(conj12(F3), F1, F1, negx=True))
    unscale(F1)
    # F3 = frob2(Bv) conj(Bv) (conj's signs on F3's reads); F2 = m^3 F3; Bv re-stored (a product-free
    # copy round: its negated shadows are written there, just before the chain's first squaring reads
    # them, instead of living from Bv's product through these rounds); F3 = e(Bv); F1 = e(F3); r = F1 F2
    p.round(frob_ops(p, F1, 2, F3))
    p.round(fp12_mul_ops(F3, conj12(F1), F3, negx=True))
    p.round(fp12_mul_ops(F3, F2, F2, negx=True))
    p.round(copy_ops(flat12(F1), flat12(F1)))
    exp_x(F1, F3)
    unscale(F3)
    exp_x(F3, F1)
    p.round(fp12_mul_ops(F1, F2, F2, negx=True))
    unscale(F2)
    for i in range(6):
        for c in range(2):
            p.named[f"r{i}_{c}"] = F2[i][c].slot
    return p


# ============================================================================ hash_to_G2 tail
# 3-isogeny E2' -> E2 of RFC 9380 (App. E.3): coefficients of x_num, x_den, y_num, y_den (lowest degree
# first, Fp2 pairs (c0, c1); the top coefficient of each denominator is 1)
ISO_XNUM = [
    (0x5C759507E8E333EBB5B7A9A47D7ED8532C52D39FD3A042A88B58423C50AE15D5C2638E343D9C71C6238AAAAAAAA97D6,
     0x5C759507E8E333EBB5B7A9A47D7ED8532C52D39FD3A042A88B58423C50AE15D5C2638E343D9C71C6238AAAAAAAA97D6),
    (0, 0x11560BF17BAA99BC32126FCED787C88F984F87ADF7AE0C7F9A208C6B4F20A4181472AAA9CB8D555526A9FFFFFFFFC71A),
    (0x11560BF17BAA99BC32126FCED787C88F984F87ADF7AE0C7F9A208C6B4F20A4181472AAA9CB8D555526A9FFFFFFFFC71E,
     0x8AB05F8BDD54CDE190937E76BC3E447CC27C3D6FBD7063FCD104635A790520C0A395554E5C6AAAA9354FFFFFFFFE38D),
    (0x171D6541FA38CCFAED6DEA691F5FB614CB14B4E7F4E810AA22D6108F142B85757098E38D0F671C7188E2AAAAAAAA5ED1, 0),
]
ISO_XDEN = [(0, P - 72), (12, P - 12), (1, 0)]
ISO_YNUM = [
    (0x1530477C7AB4113B59A4C18B076D11930F7DA5D4A07F649BF54439D87D27E500FC8C25EBF8C92F6812CFC71C71C6D706,
     0x1530477C7AB4113B59A4C18B076D11930F7DA5D4A07F649BF54439D87D27E500FC8C25EBF8C92F6812CFC71C71C6D706),
    (0, 0x5C759507E8E333EBB5B7A9A47D7ED8532C52D39FD3A042A88B58423C50AE15D5C2638E343D9C71C6238AAAAAAAA97BE),
    (0x11560BF17BAA99BC32126FCED787C88F984F87ADF7AE0C7F9A208C6B4F20A4181472AAA9CB8D555526A9FFFFFFFFC71C,
     0x8AB05F8BDD54CDE190937E76BC3E447CC27C3D6FBD7063FCD104635A790520C0A395554E5C6AAAA9354FFFFFFFFE38F),
    (0x124C9AD43B6CF79BFBF7043DE3811AD0761B0F37A1E26286B0E977C69AA274524E79097A56DC4BD9E1B371C71C718B10, 0),
]
ISO_YDEN = [(P - 432, P - 432), (0, P - 216), (18, P - 18), (1, 0)]


def _iso_consts():
    return ISO_XNUM, ISO_XDEN, ISO_YNUM, ISO_YDEN


class G2Ops:
    """Complete projective formulas on E2: y^2 = x^3 + 4(1 + u) (Renes-Costello-Batina 2016, a = 0,
    b3 = 12(1 + u)) as SOP rounds: exact for every input (identity, P + P, P - P), so hash_to_G2 needs no
    branches.  Points are (X, Y, Z) of Fp2 views; negation and psi's conjugations are views."""

    def __init__(self, p):
        self.p = p
        self.t = [slots2(p) for _ in range(6)]   # round-1 products (round 2 overwrites them in place)
        self.u = None
        self.one = T(p.const(1))

    def dbl(self, P, out):
        """out = 2P (RCB Alg. 9, a = 0) scaled by 3, which leaves the projective point unchanged:
        with t0 = Y^2, t1 = YZ, w = 3 b3 Z^2 = 36 xi Z^2 and XY,
            X3 = 6 XY (t0 - w),  Y3 = 3 (t0 + w)^2 - 4 w^2,  Z3 = 24 t0 t1
        (RCB's X3 = 2 XY (t0 - 3 t2), Y3 = t0^2 + 6 t0 t2 - 3 t2^2, Z3 = 8 t0 t1 with t2 = b3 Z^2, times 3).
        Two rounds (8 ops of <= 2 products, then 6 ops of <= 3); `out` may be P (in place)."""
        p = self.p
        X, Y, Z = P
        t0, t1, w, xy = self.t[:4]
        p.round([Op(dst_of(t0[c]), fp2_sqr(Y, c)) for c in range(2)] +
                [Op(dst_of(t1[c]), fp2_prod(Y, Z, c)) for c in range(2)] +
                [Op(dst_of(w[c]), fp2_sqr(Z, c, xi=True, m=36)) for c in range(2)] +
                [Op(dst_of(xy[c]), fp2_prod(X, Y, c)) for c in range(2)])
        (a0, a1), (w0, w1), (x0, x1) = t0, w, xy
        d0, d1 = [a0, ~w0], [a1, ~w1]            # t0 - w
        s0, s1 = [a0, w0], [a1, w1]              # t0 + w
        ops = [Op(dst_of(out[0][0]), [(d0, [x0], 6), (d1, [x1], -6)]),
               Op(dst_of(out[0][1]), [(d0, [x1], 6), (d1, [x0], 6)]),
               Op(dst_of(out[1][0]), [(s0, s0, 3), (s1, s1, -3), ([w0, w1], [w0, ~w1], -4)]),
               Op(dst_of(out[1][1]), [(s0, s1, 6), ([w0], [w1], -8)])]
        ops += [Op(dst_of(out[2][c]), fp2_prod(t0, t1, c, m=24)) for c in range(2)]
        p.round(ops)

    def add(self, P1, P2, out):
        """out = P1 + P2 (RCB Alg. 7): three rounds (12, 8, 6 lanes); `out` may be P1 or P2."""
        p = self.p
        X1, Y1, Z1 = P1
        X2, Y2, Z2 = P2
        t0, t1, t2, t3, t4, y3 = self.t
        ops = [Op(dst_of(t0[c]), fp2_prod(X1, X2, c)) for c in range(2)]
        ops += [Op(dst_of(t1[c]), fp2_prod(Y1, Y2, c)) for c in range(2)]
        ops += [Op(dst_of(t2[c]), fp2_prod(Z1, Z2, c)) for c in range(2)]
        ops += [Op(dst_of(t3[c]), fp2_prod(X1, Y2, c) + fp2_prod(Y1, X2, c)) for c in range(2)]
        ops += [Op(dst_of(t4[c]), fp2_prod(Y1, Z2, c) + fp2_prod(Z1, Y2, c)) for c in range(2)]
        ops += [Op(dst_of(y3[c]), fp2_prod(X1, Z2, c) + fp2_prod(Z1, X2, c)) for c in range(2)]
        p.round(ops)
        # round 2 writes over round 1's values in place (every read of a round precedes its stores):
        # z3 over t1, t1m over t2, y3b over y3, x3t over t0 — no separate temporaries (r04)
        z3, t1m, y3b, x3t = (t1, t2, y3, t0) if self.u is None else self.u
        one = self.one
        # b3 v = 12 (1 + u) v: (12 v0 - 12 v1, 12 v0 + 12 v1)
        p.round([Op(dst_of(z3[0]), [([t1[0]], [one], 1)], [(t2[0].slot, 12), (t2[1].slot, -12)]),
                 Op(dst_of(z3[1]), [([t1[1]], [one], 1)], [(t2[0].slot, 12), (t2[1].slot, 12)]),
                 Op(dst_of(t1m[0]), [([t1[0]], [one], 1)], [(t2[0].slot, -12), (t2[1].slot, 12)]),
                 Op(dst_of(t1m[1]), [([t1[1]], [one], 1)], [(t2[0].slot, -12), (t2[1].slot, -12)]),
                 Op(dst_of(y3b[0]), [], [(y3[0].slot, 12), (y3[1].slot, -12)]),
                 Op(dst_of(y3b[1]), [], [(y3[0].slot, 12), (y3[1].slot, 12)]),
                 Op(dst_of(x3t[0]), [], [(t0[0].slot, 3)]),
                 Op(dst_of(x3t[1]), [], [(t0[1].slot, 3)])])
        ops = [Op(dst_of(out[0][c]), fp2_prod(t3, t1m, c) + fp2_prod(t4, y3b, c, m=-1)) for c in range(2)]
        ops += [Op(dst_of(out[1][c]), fp2_prod(y3b, x3t, c) + fp2_prod(t1m, z3, c)) for c in range(2)]
        ops += [Op(dst_of(out[2][c]), fp2_prod(z3, t4, c) + fp2_prod(x3t, t3, c)) for c in range(2)]
        p.round(ops)

    def mul_xabs(self, P, out):
        """out = [|x|]P (out must not alias P)."""
        first = True
        for bit in bin(X_ABS)[3:]:
            self.dbl(P if first else out, out)
            first = False
            if bit == "1":
                self.add(out, P, out)

    def psi(self, P, out):
        """psi(X : Y : Z) = (conj(X) cx : conj(Y) cy : conj(Z)); the conj(Z) is a view of `out`'s Z."""
        p = self.p
        X, Y, Z = P
        cx = (T(p.const(PSI_CX[0])), T(p.const(PSI_CX[1])))
        cy = (T(p.const(PSI_CY[0])), T(p.const(PSI_CY[1])))
        ops = [Op(dst_of(out[0][c]), fp2_prod((X[0], ~X[1]), cx, c)) for c in range(2)]
        ops += [Op(dst_of(out[1][c]), fp2_prod((Y[0], ~Y[1]), cy, c)) for c in range(2)]
        ops += copy_ops([Z[0], ~Z[1]], list(out[2]))
        p.round(ops)


def g2_neg_view(P):
    return (P[0], neg2(P[1]), P[2])


def g2_slots(p, name=None):
    return tuple(slots2(p, f"{name}{c}" if name else None) for c in "xyz")


def h2c_program(team=8):
    """hash_to_G2 after the two SSWU maps (inputs: the affine E2' points m0, m1): 3-isogeny to E2 in
    projective form (xn yd : y yn xd : xd yd), Q0 + Q1, clear_cofactor (RFC 9380 App. G.3:
    [x^2 - x - 1]P + [x - 1] psi(P) + psi^2(2P)), then affine (hx, hy) and hz."""
    p = Program("h2c", team)
    XN, XD, YN, YD = _iso_consts()
    m = [(slots2(p, f"m{k}x"), slots2(p, f"m{k}y")) for k in range(2)]
    x2 = [slots2(p) for _ in range(2)]
    x3 = [slots2(p) for _ in range(2)]
    # powers of x
    p.round([Op(dst_of(x2[k][c]), fp2_sqr(m[k][0], c)) for k in range(2) for c in range(2)])
    p.round([Op(dst_of(x3[k][c]), fp2_prod(x2[k], m[k][0], c)) for k in range(2) for c in range(2)])
    cst = lambda v: (T(p.const(v[0])), T(p.const(v[1])))  # noqa: E731

    def poly_ops(k, cs, dst):
        """sum_i cs[i] x^i with a monic top term (cs[-1] == (1, 0)) taken as an add-in."""
        xp = {1: m[k][0], 2: x2[k], 3: x3[k]}
        deg = len(cs) - 1
        ops = []
        for c in range(2):
            prods, adds = [], []
            for i in range(1, deg + 1):
                if cs[i] == (1, 0):
                    adds.append((xp[i][c].slot, 1))
                elif cs[i] != (0, 0):
                    prods += fp2_prod(cst(cs[i]), xp[i], c)
            c0 = cs[0][c]
            if c0:
                adds.append((p.const(c0), 1))
            assert len(adds) <= 2
            ops.append(Op(dst_of(dst[c]), prods, adds))
        return ops
    xn, xd, yn, yd = ([slots2(p) for _ in range(2)] for _ in range(4))
    p.round([o for k in range(2) for o in poly_ops(k, XN, xn[k]) + poly_ops(k, YN, yn[k])] +
            [o for k in range(2) for o in poly_ops(k, XD, xd[k])])
    p.round([o for k in range(2) for o in poly_ops(k, YD, yd[k])])
    # (r04) the isogeny's temporaries are released as they die, so the points reuse their slots
    p.release([v.slot for grp in (x2, x3) for f2 in grp for v in f2] + [v.slot for pt in m for v in pt[0]])
    q = [g2_slots(p) for _ in range(2)]
    yyn = [slots2(p) for _ in range(2)]
    p.round([Op(dst_of(q[k][0][c]), fp2_prod(xn[k], yd[k], c)) for k in range(2) for c in range(2)] +
            [Op(dst_of(q[k][2][c]), fp2_prod(xd[k], yd[k], c)) for k in range(2) for c in range(2)] +
            [Op(dst_of(yyn[k][c]), fp2_prod(m[k][1], yn[k], c)) for k in range(2) for c in range(2)])
    p.round([Op(dst_of(q[k][1][c]), fp2_prod(yyn[k], xd[k], c)) for k in range(2) for c in range(2)])
    p.release([v.slot for grp in (xn, xd, yn, yd, yyn) for f2 in grp for v in f2] +
              [v.slot for pt in m for v in pt[1]])
    g = G2Ops(p)
    Pt = g2_slots(p)
    g.add(q[0], q[1], Pt)
    # clear_cofactor (RFC 9380 G.3): Q = [x^2 - x - 1] Pt + [x - 1] psi(Pt) + psi^2(2 Pt), with A = [|x|] Pt:
    #   t2 = psi(Pt);  t3 = psi^2(2 Pt) - t2;  t3 = (A + t3) ... u = Pt - t3;  t2 = t2 - A;  -Q = u + [|x|] t2
    # (r04 order) the psi terms first, then the chains; every addition takes the value it just made as P1
    # (its negated reads land on that value's shadows) and Pt / A die before the second chain
    t2 = q[0]                       # q0, q1 are dead after Pt
    g.psi(Pt, t2)
    t3 = q[1]
    g.dbl(Pt, t3)
    g.psi(t3, t3)
    g.psi(t3, t3)
    g.add(t3, g2_neg_view(t2), t3)
    A = g2_slots(p)
    g.mul_xabs(Pt, A)
    g.add(A, t3, t3)
    g.add(g2_neg_view(t3), Pt, t3)  # u = Pt - (psi^2(2 Pt) - psi(Pt) + A)
    g.add(g2_neg_view(A), t2, t2)   # t2 = psi(Pt) - A
    p.release([v.slot for pt in (Pt, A) for f2 in pt for v in f2])
    B = g2_slots(p)
    g.mul_xabs(t2, B)
    g.add(B, t3, t3)                 # w = u + [|x|] t2 = -Q
    p.release([v.slot for pt in (t2, B) for f2 in pt for v in f2] + [v.slot for f2 in g.t for v in f2])
    X, Y, Z = g2_neg_view(t3)
    # affine: zi = Z^-1 via the norm
    n, ninv = T(p.alloc()), T(p.alloc())
    p.round([Op(n.slot, [([Z[0]], [Z[0]], 1), ([Z[1]], [Z[1]], 1)])])
    p.round([Op(ninv.slot, [], [(n.slot, 1)], kind="inv")])
    zi = slots2(p)
    p.round([Op(dst_of(zi[0]), [([Z[0]], [ninv], 1)]), Op(dst_of(zi[1]), [([Z[1]], [ninv], -1)])])
    hx, hy, hz = slots2(p, "hx"), slots2(p, "hy"), slots2(p, "hz")
    p.round([Op(dst_of(hx[c]), fp2_prod(X, zi, c)) for c in range(2)] +
            [Op(dst_of(hy[c]), fp2_prod(Y, zi, c)) for c in range(2)] + copy_ops(list(Z), list(hz)))
    return p


def check_h2c(hp):
    from oracle import bls12_381 as B
    rnd = random.Random(11)
    for _ in range(2):
        msg = rnd.randbytes(32)
        u = B.hash_to_field_fp2(msg, 2, B.DST_POP)
        mem = {s: 0 for s in range(hp.nslots)}
        for k in range(2):
            x, y = B.sswu_g2(u[k])
            for nm, v in ((f"m{k}x0", x[0]), (f"m{k}x1", x[1]), (f"m{k}y0", y[0]), (f"m{k}y1", y[1])):
                mem[hp.named[nm]] = mont(v)
        hp.emulate(mem)
        got = ((unmont(mem[hp.named["hx0"]]), unmont(mem[hp.named["hx1"]])),
               (unmont(mem[hp.named["hy0"]]), unmont(mem[hp.named["hy1"]])))
        assert got == B.hash_to_g2(msg), "SOP h2c mismatch"
        assert mem[hp.named["hz0"]] or mem[hp.named["hz1"]]
    print("  SOP hash_to_G2 tail checked against the oracle")


# ============================================================================ checks against the oracle
def _f12_from_mem(p, mem, name):
    g = [(unmont(mem[p.named[f"{name}{i}_0"]]), unmont(mem[p.named[f"{name}{i}_1"]])) for i in range(6)]
    return g


def _line_inputs(lp, pt, q):
    mem = {}
    (qx0, qx1), (qy0, qy1) = q
    for nm, v in (("qx0", qx0), ("qx1", qx1), ("qy0", qy0), ("qy1", qy1), ("tx0", qx0), ("tx1", qx1),
                  ("ty0", qy0), ("ty1", qy1), ("tz0", 1), ("tz1", 0), ("nxp", (-pt[0]) % P), ("yp", pt[1])):
        mem[lp.named[nm]] = mont(v)
    for s in range(lp.nslots):
        mem.setdefault(s, 0)
    return mem


def subgroup_emulated(lp, q):
    mem = _line_inputs(lp, (1, 2), q)
    lp.emulate(mem, io_out={})
    e = [mem[lp.named[k]] for k in ("e10", "e11", "e20", "e21")]
    z = [mem[lp.named[k]] for k in ("tz0", "tz1")]
    return any(z) and not any(e)


def run_miller(lp, ap, Pp, Q):
    """Emulate: both line programs, then the accumulation; returns the Fp12 coefficients (canonical)."""
    lines = {}
    for k, (pt, q) in enumerate(zip(Pp, Q)):
        mem = _line_inputs(lp, pt, q)
        out = {}
        lp.emulate(mem, io_out=out)
        for idx, v in out.items():
            lines[6 * lp.nsteps * k + idx] = v
    mem = {s: 0 for s in range(ap.nslots)}
    mem[ap.named["f0_0"]] = mont(1)
    ap.emulate(mem, io_in=lines)
    return _f12_from_mem(ap, mem, "f")


def check_miller(lp, ap):
    from oracle import bls12_381 as B
    rnd = random.Random(7)
    for _ in range(2):
        a, b = rnd.randrange(1, 1 << 60), rnd.randrange(1, 1 << 60)
        P1 = B.g1_mul(B.G1_GEN, a)
        Q1 = B.g2_mul(B.G2_GEN, b)
        Q2 = B.g2_mul(B.G2_GEN, b + 7)
        P2 = B.g1_neg(B.G1_GEN)
        g = run_miller(lp, ap, [P1, P2], [Q1, Q2])
        got = B.final_exponentiation(B.f12_from_coeffs(g))
        exp = B.f12_mul(B.pairing(P1, Q1), B.pairing(P2, Q2))
        assert got == exp, "SOP miller mismatch"
    # the fused G2 subgroup check: members and non-members of G2
    cases = [(B.g2_mul(B.G2_GEN, rnd.randrange(1, B.R)), True)]
    x = 1
    while len(cases) < 4:
        x += 1
        X = (x, 5)
        y = B.f2_sqrt(B.f2_add(B.f2_mul(B.f2_sqr(X), X), B.B2))
        if y is not None:
            cases.append(((X, y), False))
    # the exceptional path (tests/g2_edge_points.py): points of the cofactor's small
    # orders (order 13 meets T = -Q before the walk's second addition), G2 + torsion sums
    g = B.g2_mul(B.G2_GEN, rnd.randrange(1, B.R))
    for ell in (13, 23, 2713, 11953, 262069):
        t = B.g2_point_of_order(ell)
        cases += [(t, False), (B.g2_neg(t), False), (B.g2_add(g, t), False)]
    cases.append((B.g2_point_of_order(B.H2_BIG), False))
    for q, want in cases:
        assert subgroup_emulated(lp, q) == want == B.g2_in_subgroup(q), "SOP subgroup check mismatch"
    print("  SOP Miller (lines + accumulation) checked against oracle pairings; fused G2 subgroup check too "
          f"({len(cases)} points, incl. small-order / G2 + torsion points)")


def run_miller_fused(mp, Pp, Q):
    """Emulate the fused program (miller_program): m_ walk = pairing 0, s_ walk = pairing 1; returns the
    Fp12 coefficients and the signature walk's subgroup verdict."""
    mem = {s: 0 for s in range(mp.nslots)}
    for k, prefix in ((0, "m_"), (1, "s_")):
        (qx0, qx1), (qy0, qy1) = Q[k]
        pt = Pp[k]
        for nm, v in (("qx0", qx0), ("qx1", qx1), ("qy0", qy0), ("qy1", qy1), ("tx0", qx0), ("tx1", qx1),
                      ("ty0", qy0), ("ty1", qy1), ("tz0", 1), ("tz1", 0), ("nxp", (-pt[0]) % P), ("yp", pt[1])):
            mem[mp.named[prefix + nm]] = mont(v)
    mem[mp.named["f0_0"]] = mont(1)
    mp.emulate(mem)
    e = [mem[mp.named["s_" + k]] for k in ("e10", "e11", "e20", "e21")]
    z = [mem[mp.named["s_" + k]] for k in ("tz0", "tz1")]
    return _f12_from_mem(mp, mem, "f"), bool(any(z) and not any(e))


def check_miller_fused(lp, ap, mp):
    from oracle import bls12_381 as B
    rnd = random.Random(17)
    for _ in range(2):
        a, b = rnd.randrange(1, 1 << 60), rnd.randrange(1, 1 << 60)
        Pp = [B.g1_mul(B.G1_GEN, a), B.g1_neg(B.G1_GEN)]
        Q = [B.g2_mul(B.G2_GEN, b), B.g2_mul(B.G2_GEN, b + 11)]
        g, ok = run_miller_fused(mp, Pp, Q)
        assert g == run_miller(lp, ap, Pp, Q), "fused Miller program differs from lines + accumulation"
        assert ok, "fused subgroup check rejected a G2 point"
    bad = B.g2_add(B.g2_mul(B.G2_GEN, 5), B.g2_point_of_order(13))
    g, ok = run_miller_fused(mp, [B.g1_neg(B.G1_GEN), B.g1_neg(B.G1_GEN)], [B.g2_mul(B.G2_GEN, 3), bad])
    assert not ok and not B.g2_in_subgroup(bad), "fused subgroup check accepted a non-member"
    print("  SOP fused Miller program (both walks beside the accumulation) equals lines + accumulation; "
          "its subgroup check rejects a G2 + torsion point")


def check_fexp(fp):
    from oracle import bls12_381 as B
    rnd = random.Random(9)
    f = tuple(tuple((rnd.randrange(P), rnd.randrange(P)) for _ in range(3)) for _ in range(2))
    g = B.f12_coeffs(f)
    mem = {s: 0 for s in range(fp.nslots)}
    for i in range(6):
        mem[fp.named[f"f{i}_0"]], mem[fp.named[f"f{i}_1"]] = mont(g[i][0]), mont(g[i][1])
    fp.emulate(mem)
    out = _f12_from_mem(fp, mem, "r")
    e = B.final_exponentiation(f)
    assert B.f12_from_coeffs(out) == B.f12_mul(B.f12_mul(e, e), e), "SOP fexp mismatch"
    print("  SOP final exponentiation checked against the oracle (e^3)")


# ============================================================================ emit
def emit(progs, path):
    lines = ["// GENERATED by tools/gen_sop.py — do not edit.  SOP team programs (see lcv_sop.hpp).",
             "#pragma once", "#include <stdint.h>", ""]
    schoolbook = 0
    for p in progs:
        hdr, rec = p.encode()
        # a round with products but without the Karatsuba flag needs the device's schoolbook scans
        schoolbook |= any((w0 & 15) and not (w0 >> 22) & 1 for w0 in hdr[0::4])
        N = p.name.upper()
        lines.append(f"// {p.stats()}")
        lines.append(f"#define LCV_SOP_{N}_TEAM {p.team}")
        lines.append(f"#define LCV_SOP_{N}_ROUNDS {len(hdr) // 4}")
        lines.append(f"#define LCV_SOP_{N}_SLOTS {p.nslots}")
        lines.append(f"#define LCV_SOP_{N}_NCONST {len(p.consts)}")
        lines.append(f"#define LCV_SOP_{N}_MAXK {max(max(len(o.prods) for o in r) for r in p.rounds)}")
        if hasattr(p, "nsteps"):
            lines.append(f"#define LCV_SOP_{N}_NSTEPS {p.nsteps}")
        for nm, s in sorted(p.named.items(), key=lambda kv: kv[1]):
            lines.append(f"#define LCV_SOP_{N}_SLOT_{nm.upper()} {s}")
        lines.append(f"static const uint32_t kSop_{p.name}_hdr[{len(hdr)}] = {{")
        for i in range(0, len(hdr), 16):
            lines.append("  " + ",".join(str(w) for w in hdr[i:i + 16]) + ",")
        lines.append("};")
        lines.append(f"static const uint32_t kSop_{p.name}_rec[{len(rec)}] = {{")
        for i in range(0, len(rec), 16):
            lines.append("  " + ",".join(str(w) for w in rec[i:i + 16]) + ",")
        lines.append("};")
        lines.append(f"static const uint32_t kSop_{p.name}_consts[{max(1, len(p.consts)) * 12}] = {{")
        for c in p.const_list() or [0]:
            mv = mont(c)
            lines.append("  " + ",".join(f"0x{(mv >> (32 * k)) & 0xffffffff:08x}u" for k in range(12)) + ",")
        lines.append("};")
        lines.append("")
    lines.append("// 1: some product round of these programs is not Karatsuba-eligible (14 x 14 / 15 x 14 schoolbook)")
    lines.append(f"#define LCV_SOP_SCHOOLBOOK {int(schoolbook)}")
    open(path, "w").write("\n".join(lines) + "\n")


def build():
    global PSI_CX, PSI_CY
    PSI_CX, PSI_CY = _psi_consts()
    lp = line_program()
    ap = acc_program(nsteps=lp.nsteps)
    fp = fexp_program()
    hp = h2c_program()
    mp = miller_program()
    progs = (lp, ap, fp, hp, mp)
    perms = os.environ.get("LCV_SOP_SLOT_PERMS")  # experiment: JSON {program: perm}
    if perms:
        import json
        for p, perm in json.load(open(perms)).items():
            prog = {q.name: q for q in progs}[p]
            prog.finalize()
            prog.relabel(perm)
    return progs


def main():
    ap_ = argparse.ArgumentParser()
    ap_.add_argument("--check", action="store_true")
    ap_.add_argument("--out", default=os.path.join(ROOT, "light-client-consensus-specs_amd", "csrc",
                                                  "lcv_sop_programs.inc"))
    args = ap_.parse_args()
    progs = build()
    for p in progs:
        p.finalize()
        print(p.stats())
    if args.check:
        check_miller(progs[0], progs[1])
        check_miller_fused(progs[0], progs[1], progs[4])
        check_fexp(progs[2])
        check_h2c(progs[3])
    emit(progs, args.out)


if __name__ == "__main__":
    main()
