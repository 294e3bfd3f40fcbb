#!/usr/bin/env python3
"""Writes csrc/xm_pk_taps.h: the packed-tap asm blocks of the fast kernel
(csrc/xm_resample_fast.hip, TAPS == 2), one block per 8-tap coefficient group
(G0, G1: 8 taps; G2: the 6-tap last group of 48k->44.1k, G2T5 / G2T4: the 5- and
4-tap last groups of 44.1k->48k).

Operands of every block: %0..%3 product temps (=&v), %4 a0, %5 a1 (+v, the
(L, R) accumulators of outputs k, k+1), %6..%13 coefficient SGPR pairs
(h_k[t], h_k+1[t]) of the group, %14.. the window pairs: x[ra+t], x[rb+t] per
tap (single-output blocks: x[ra+t] only).  Products of tap t+1 are issued before
the adds of tap t (two temp pairs alternate), the adds stay in tap order, so the
arithmetic is exactly the ascending-t chain of the contract.
"""
import os

def block(ntaps, first, two):
    lines = []
    def mul(t):
        tp = 2 * (t % 2)
        c = 6 + t
        xa = 14 + (2 * t if two else t)
        if first and t == 0:   # tap 0 initialises the accumulators
            lines.append(f"v_pk_mul_f32 %4, %{c}, %{xa} op_sel_hi:[0,1]")
            if two:
                lines.append(f"v_pk_mul_f32 %5, %{c}, %{xa + 1} op_sel:[1,0] op_sel_hi:[1,1]")
            return
        lines.append(f"v_pk_mul_f32 %{tp}, %{c}, %{xa} op_sel_hi:[0,1]")
        if two:
            lines.append(f"v_pk_mul_f32 %{tp + 1}, %{c}, %{xa + 1} op_sel:[1,0] op_sel_hi:[1,1]")
    def add(t):
        if first and t == 0:
            return
        tp = 2 * (t % 2)
        lines.append(f"v_pk_add_f32 %4, %4, %{tp}")
        if two:
            lines.append(f"v_pk_add_f32 %5, %5, %{tp + 1}")
    mul(0)
    for t in range(1, ntaps):
        mul(t)
        add(t - 1)
    add(ntaps - 1)
    return "\\n\\t".join(lines)

def vblock(ntaps, first, two):
    """VOP2 taps with literal coefficients (TAPS == 1).  Operands: %0..%7
    product temps (=&v; two sets alternate so tap t+1's products issue before
    tap t's adds), accumulators %8..%11 = l0 r0 l1 r1 (+v, =&v when `first`),
    then per tap t: h_k, h_k+1 ("i" bit patterns), xl[ra+t], xr[ra+t],
    xl[rb+t], xr[rb+t].  Single-output blocks: temps %0..%3, accumulators
    %4 %5 = l0 r0, per tap: h_k, xl[ra+t], xr[ra+t]."""
    lines = []
    if two:
        acc, nt, per = 8, 4, 6
    else:
        acc, nt, per = 4, 2, 3
    ntemp_base = 0
    def ops(t):
        b = acc + (4 if two else 2) + per * t
        if two:
            return dict(h0=b, h1=b + 1, xla=b + 2, xra=b + 3, xlb=b + 4, xrb=b + 5)
        return dict(h0=b, xla=b + 1, xra=b + 2)
    def mul(t):
        o = ops(t)
        dst = [acc + i for i in range(nt)] if (first and t == 0) else [ntemp_base + nt * (t % 2) + i for i in range(nt)]
        lines.append(f"v_mul_f32 %{dst[0]}, %{o['h0']}, %{o['xla']}")
        lines.append(f"v_mul_f32 %{dst[1]}, %{o['h0']}, %{o['xra']}")
        if two:
            lines.append(f"v_mul_f32 %{dst[2]}, %{o['h1']}, %{o['xlb']}")
            lines.append(f"v_mul_f32 %{dst[3]}, %{o['h1']}, %{o['xrb']}")
    def add(t):
        if first and t == 0:
            return
        for i in range(nt):
            lines.append(f"v_add_f32 %{acc + i}, %{acc + i}, %{nt * (t % 2) + i}")
    mul(0)
    for t in range(1, ntaps):
        mul(t)
        add(t - 1)
    add(ntaps - 1)
    return "\\n\\t".join(lines)

# SGPR pairs the literal-coefficient blocks load (clobbered by every block)
LK_SGPR = (96, 98)


def lblock(ntaps, first, two):
    """Packed taps with literal coefficients (the LIT kernels, 320/147: the
    pair table does not fit the scalar cache): no scalar memory.
    Per tap t the coefficient pair (h_k[t], h_k+1[t]) is written into an SGPR
    pair by two s_mov_b32 (SALU, issued between the VALU of the previous tap;
    the two pairs alternate by tap parity) and read by the two v_pk_mul_f32
    exactly as the SGPR-pair operand of the TAPS == 2 blocks.  Operands: %0..%3
    product temps (=&v), %4 a0, %5 a1 (accumulators), then per tap: h_k, h_k+1
    ("i" bit patterns), x[ra+t], x[rb+t] (single-output blocks: h_k, x[ra+t])."""
    lines = []
    per = 4 if two else 2
    def ops(t):
        b = 6 + per * t
        return (b, b + 1, b + 2, b + 3) if two else (b, None, b + 1, None)
    def movs(t):
        h0, h1, _, _ = ops(t)
        sp = LK_SGPR[t % 2]
        lines.append(f"s_mov_b32 s{sp}, %{h0}")
        if two:
            lines.append(f"s_mov_b32 s{sp + 1}, %{h1}")
    def mul(t):
        _, _, xa, xb = ops(t)
        sp = LK_SGPR[t % 2]
        tp = 2 * (t % 2)
        if first and t == 0:
            lines.append(f"v_pk_mul_f32 %4, s[{sp}:{sp + 1}], %{xa} op_sel_hi:[0,1]")
            if two:
                lines.append(f"v_pk_mul_f32 %5, s[{sp}:{sp + 1}], %{xb} op_sel:[1,0] op_sel_hi:[1,1]")
            return
        lines.append(f"v_pk_mul_f32 %{tp}, s[{sp}:{sp + 1}], %{xa} op_sel_hi:[0,1]")
        if two:
            lines.append(f"v_pk_mul_f32 %{tp + 1}, s[{sp}:{sp + 1}], %{xb} op_sel:[1,0] op_sel_hi:[1,1]")
    def add(t):
        if first and t == 0:
            return
        tp = 2 * (t % 2)
        lines.append(f"v_pk_add_f32 %4, %4, %{tp}")
        if two:
            lines.append(f"v_pk_add_f32 %5, %5, %{tp + 1}")
    movs(0)
    mul(0)
    for t in range(1, ntaps):
        movs(t)
        mul(t)
        add(t - 1)
    add(ntaps - 1)
    return "\\n\\t".join(lines)


out = ["// generated by tools/gen_pk_asm.py; do not edit", "#pragma once"]
for n in range(1, 5):
    for first in (True, False):
        for two in (True, False):
            out.append(f'#define XM_V2_{"F" if first else "R"}{n}_{"TWO" if two else "ONE"} "{vblock(n, first, two)}"')
# G2T<n>: an n-tap last group (1..7 taps: every ratio's T mod 8)
for first, n, name in ((True, 8, "G0"), (False, 8, "G1"), (False, 6, "G2")) + tuple(
        (False, n, f"G2T{n}") for n in (1, 2, 3, 4, 5, 7)):
    for two in (True, False):
        out.append(f'#define XM_PK_{name}_{"TWO" if two else "ONE"} "{block(n, first, two)}"')
for n in (1, 2, 3, 4):
    for first in (True, False):
        for two in (True, False):
            if first and n != 4:
                continue
            out.append(f'#define XM_LK_{"F" if first else "R"}{n}_{"TWO" if two else "ONE"} "{lblock(n, first, two)}"')
out.append(f'#define XM_LK_CLOBBER "s{LK_SGPR[0]}", "s{LK_SGPR[0] + 1}", "s{LK_SGPR[1]}", "s{LK_SGPR[1] + 1}"')
path = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "csrc", "xm_pk_taps.h")
open(path, "w").write("\n".join(out) + "\n")
