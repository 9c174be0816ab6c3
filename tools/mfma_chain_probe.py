#!/usr/bin/env python3
"""tools/mfma_chain_probe.py -- which arithmetic does a 16x16x4 matrix-core instruction perform?  

The engine's matrix-core tiles are bit-identical to the reference only if the instruction is the reference's own
operation sequence: C[r][j] = fma(a_3, b_3, fma(a_2, b_2, fma(a_1, b_1, fma(a_0, b_0, C[r][j])))) -- k in order, one
rounding per step (the reference's `sum += a*x` contracted by GCC, spmm_kernel_csr.cpp:87-91).  For random operands
of mixed signs and magnitudes (so the candidates round differently) this runs v_mfma_f64_16x16x4f64 and
v_mfma_f32_16x16x4f32 once per problem (tools/mfma_chain_probe.hip) and counts, per instruction, the outputs equal
bit for bit to each candidate computed exactly on the host (rationals):
  chain_asc   the fma chain, k = 0, 1, 2, 3
  chain_desc  the fma chain, k = 3, 2, 1, 0
  fused_dot   C + a_0 b_0 + ... + a_3 b_3 rounded once
  prod_tree   products rounded, then ((p0 + p1) + (p2 + p3)) + C, each addition rounded
Prints one JSON line per dtype.  The f32 matrix tiles are only worth building if chain_asc matches every output.

  python tools/mfma_chain_probe.py --problems 200
"""
import argparse
import ctypes
import json
import sys
from fractions import Fraction
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
LIB = ROOT / "spmm-research_amd" / "lib" / "libmfma_chain_probe.so"


def round_to(q: Fraction, mant: int) -> Fraction:
    """Round a rational to the nearest binary float with `mant` fraction bits (ties to even); normal range only."""
    if q == 0:
        return Fraction(0)
    s = -1 if q < 0 else 1
    q = abs(q)
    e = q.numerator.bit_length() - q.denominator.bit_length()
    if Fraction(2) ** e > q:
        e -= 1
    elif Fraction(2) ** (e + 1) <= q:
        e += 1
    m = q / Fraction(2) ** (e - mant)
    n = m.numerator // m.denominator
    r = m - n
    if r > Fraction(1, 2) or (r == Fraction(1, 2) and n % 2 == 1):
        n += 1
    return s * n * Fraction(2) ** (e - mant)


def candidates(a, b, c, mant):
    F = [Fraction(float(x)) for x in a], [Fraction(float(x)) for x in b]
    C0 = Fraction(float(c))
    p = [F[0][k] * F[1][k] for k in range(4)]
    out = {}
    x = C0
    for k in range(4):
        x = round_to(p[k] + x, mant)
    out["chain_asc"] = x
    x = C0
    for k in (3, 2, 1, 0):
        x = round_to(p[k] + x, mant)
    out["chain_desc"] = x
    out["fused_dot"] = round_to(C0 + sum(p), mant)
    pr = [round_to(v, mant) for v in p]
    out["prod_tree"] = round_to(round_to(round_to(pr[0] + pr[1], mant) + round_to(pr[2] + pr[3], mant), mant) + C0, mant)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--problems", type=int, default=200)
    ap.add_argument("--seed", type=int, default=1)
    args = ap.parse_args()
    import torch
    L = ctypes.CDLL(str(LIB))
    L.chain_probe.argtypes = [ctypes.c_int] + [ctypes.c_void_p] * 4 + [ctypes.c_int, ctypes.c_void_p]
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(args.seed)
    n = args.problems
    for f64, dt, mant in ((1, np.float64, 52), (0, np.float32, 23)):
        def draw(shape):
            v = rng.uniform(1.0, 2.0, shape) * 2.0 ** rng.integers(-12, 12, shape) * rng.choice([-1.0, 1.0], shape)
            return v.astype(dt)
        a, b, c = draw((n, 64)), draw((n, 64)), draw((n, 64, 4))
        ta, tb, tc = (torch.from_numpy(x).to(dev) for x in (a, b, c))
        td = torch.empty_like(tc)
        st = L.chain_probe(f64, ta.data_ptr(), tb.data_ptr(), tc.data_ptr(), td.data_ptr(), n,
                           torch.cuda.current_stream(dev).cuda_stream)
        assert st == 0, st
        torch.cuda.synchronize()
        d = td.cpu().numpy()
        # operand layout (16x16x4): lane l holds A[l & 15][l >> 4] and B[l >> 4][l & 15]; output i of lane l is
        # D[row(l, i)][l & 15] -- both row maps the instruction family uses are tried, the better one is reported
        res = {}
        for name, rowmap in (("row=(l>>4)+4i", lambda l, i: (l >> 4) + 4 * i),
                             ("row=4(l>>4)+i", lambda l, i: 4 * (l >> 4) + i)):
            hits = {h: 0 for h in ("chain_asc", "chain_desc", "fused_dot", "prod_tree")}
            total = 0
            for p in range(n):
                A = np.zeros((16, 4), dt)
                B = np.zeros((4, 16), dt)
                for l in range(64):
                    A[l & 15, l >> 4] = a[p, l]
                    B[l >> 4, l & 15] = b[p, l]
                for l in range(64):
                    for i in range(4):
                        r, j = rowmap(l, i), l & 15
                        cand = candidates(A[r, :], B[:, j], c[p, l, i], mant)
                        got = Fraction(float(d[p, l, i]))
                        total += 1
                        for h, v in cand.items():
                            hits[h] += int(v == got)
            res[name] = {"outputs": total, "match": hits}
        best = max(res, key=lambda k: res[k]["match"]["chain_asc"])
        rec = {"instruction": "v_mfma_f64_16x16x4f64" if f64 else "v_mfma_f32_16x16x4f32", "problems": n,
               "layout": best, **res[best],
               "k_ordered_fma_chain": res[best]["match"]["chain_asc"] == res[best]["outputs"]}
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    sys.exit(main())
