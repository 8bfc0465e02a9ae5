"""Correctly rounded 2^(j/256), j = 0..255, for omb_math.h (kExp2Tab256): 60-digit decimal arithmetic,
then float(Decimal) (correct rounding to the nearest double)."""
from decimal import Decimal, getcontext

getcontext().prec = 60
LN2 = Decimal(2).ln()
vals = [float((Decimal(j) / 256 * LN2).exp()) for j in range(256)]
print("__device__ constexpr double kExp2Tab256[256] = {")
for i in range(0, 256, 4):
    print("    " + ", ".join(v.hex().replace("0x1.", "0x1.").replace("p+0", "p+0") for v in vals[i:i + 4]) + ",")
print("};")
# the reduction constants of kernel_of_r2_tab256_x2 (Matern: reduce in r-space, c = ln2 / (256 √5))
c = LN2 / 256 / Decimal(5).sqrt()
c_hi = float(c)
c_lo = float(c - Decimal(c_hi))
t0 = float(-Decimal(5).sqrt() * 256 / LN2)
print("// t0 = -sqrt5*256/ln2 =", repr(t0), " c_hi =", repr(c_hi), " c_lo =", repr(c_lo))
a = []
f = Decimal(1)
for i in range(1, 5):
    f *= i
    a.append(float((-Decimal(5).sqrt()) ** i / f))
print("// a1..a4 = (-sqrt5)^i / i! =", [repr(x) for x in a])
# cross-check against the existing 64-entry table
assert all(vals[4 * j] == float((Decimal(j) / 64 * LN2).exp()) for j in range(64))
