"""Which rounding sequence does v_mfma_f64_16x16x4_f64 implement?  Reads the
probe's dump and compares D against exact-arithmetic emulations."""
import sys
from fractions import Fraction as F
import numpy as np

raw = open(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/mfma_f64.bin", "rb").read()
nt = int(np.frombuffer(raw[:4], np.int32)[0])
v = np.frombuffer(raw[4:], np.float64)
A = v[:nt * 64].reshape(nt, 16, 4); v = v[nt * 64:]
B = v[:nt * 64].reshape(nt, 4, 16); v = v[nt * 64:]
C = v[:nt * 256].reshape(nt, 16, 16); v = v[nt * 256:]
D = v[:nt * 256].reshape(nt, 16, 16)

def fma(a, b, c):
    return float(F(a) * F(b) + F(c))

def emu(kind, a, b, c):
    if kind == "fma_k_asc":
        for k in range(4): c = fma(a[k], b[k], c)
        return c
    if kind == "fma_k_desc":
        for k in (3, 2, 1, 0): c = fma(a[k], b[k], c)
        return c
    if kind == "exact_once":
        return float(sum(F(a[k]) * F(b[k]) for k in range(4)) + F(c))
    if kind == "mul_add_asc":
        for k in range(4): c = c + a[k] * b[k]
        return c
    if kind == "pair_tree":   # exact products, (p0+p1)+(p2+p3) rounded, + c
        p = [a[k] * b[k] for k in range(4)]
        return ((p[0] + p[1]) + (p[2] + p[3])) + c
    if kind == "exact_prod_sum_then_c":
        return float(F(float(sum(F(a[k]) * F(b[k]) for k in range(4)))) + F(c))

kinds = ["fma_k_asc", "fma_k_desc", "exact_once", "mul_add_asc", "pair_tree", "exact_prod_sum_then_c"]
ok = {k: 0 for k in kinds}
tot = 0
rng = np.random.default_rng(0)
for q in range(nt):
    for i in range(16):
        for j in rng.choice(16, 4, replace=False) if q >= 2 else range(16):
            a, b, c = A[q, i, :], B[q, :, j], C[q, i, j]
            tot += 1
            for k in kinds:
                if emu(k, list(map(float, a)), list(map(float, b)), float(c)) == D[q, i, j]:
                    ok[k] += 1
for k in kinds:
    print(f"{k:24s} {ok[k]}/{tot}")
