"""The sphere test's division t = x / (2a) (shapes.rs:68,75) as the device
computes it: sphere_k's per-ray reciprocal of 2a (v_rcp_f64 + two Newton steps)
finished per sphere by div_a2 with the division's own correction steps inside
an exponent window, the compiler's full f64 division outside it
(trace_common.hpp; DESIGN.md §4 "Division by 2a").  The claim is that this is
the correctly rounded quotient bit for bit; here it is checked directly,
through rt_div_a2_check, against the device's own division and numpy's
(IEEE) division on > 10^7 operand pairs: random operands, both edges of the
window (2a near 2^-100 and 2^101, |x| near 2^-900 and 2^600) and just outside,
denormals, +-0, infinities and NaNs."""
import numpy as np
import pytest

import libraytrace as lr

pytestmark = pytest.mark.gpu


def _bits_equal(p, q):
    """Bitwise equality, NaN == NaN (payloads aside)."""
    same = p.view(np.uint64) == q.view(np.uint64)
    return same | (np.isnan(p) & np.isnan(q))


def _operands(rng):
    n = 1 << 21
    # random mantissas and signs at the given biased exponents (arrays or scalars)
    def f64(exp, size):
        mant = rng.integers(0, 1 << 52, size=size, dtype=np.uint64)
        sign = rng.integers(0, 2, size=size, dtype=np.uint64) << np.uint64(63)
        e = np.broadcast_to(np.asarray(exp, dtype=np.uint64), (size,))
        return (sign | (e << np.uint64(52)) | mant).view(np.float64)
    xs, as_ = [], []
    # 1. the renders' operating point: |d|^2 ~ 1 (a2 ~ 2), x over a wide range
    xs.append(f64(rng.integers(1023 - 60, 1023 + 60, size=n), n)); as_.append(np.abs(f64(1023, n)) * rng.uniform(0.5, 2.0, n))
    # 2. a2 at and around both window edges: a = a2 / 2, a2 biased exponent 920..926 and 1120..1126
    for ea2 in list(range(920, 927)) + list(range(1120, 1127)):
        a2 = np.abs(f64(ea2, n // 8))
        xs.append(f64(rng.integers(1, 2047, size=n // 8), n // 8)); as_.append(a2 / 2.0)
    # 3. x at and around both edges of its window: biased exponent 120..126 and 1619..1625, a2 anywhere in the window
    for ex in list(range(120, 127)) + list(range(1619, 1626)):
        xs.append(f64(ex, n // 8)); as_.append(np.abs(f64(rng.integers(923, 1124, size=n // 8), n // 8)) / 2.0)
    # 4. everything at once: exponents uniform over the whole range (quotients overflow, underflow, go denormal)
    xs.append(f64(rng.integers(0, 2047, size=n), n)); as_.append(np.abs(f64(rng.integers(0, 2047, size=n), n)))
    # 5. specials for x and for a
    spec = np.array([0.0, -0.0, np.inf, -np.inf, np.nan, 5e-324, -5e-324, 2.2250738585072014e-308,
                     1.7976931348623157e308, 1.0, -1.0, 2.0 ** -900, 2.0 ** 600, np.nextafter(2.0 ** 600, 0.0),
                     np.nextafter(2.0 ** -900, 0.0)])
    gx, ga = np.meshgrid(spec, np.concatenate([np.abs(spec), [0.5, 2.0 ** -101, 2.0 ** 100, np.nextafter(2.0 ** 100, 0.0)]]))
    xs.append(gx.ravel()); as_.append(ga.ravel())
    return np.concatenate(xs), np.concatenate(as_)


def test_division_by_2a_is_ieee_bit_for_bit(gpu_ctx):
    rng = np.random.default_rng(20251018)
    x, a = _operands(rng)
    assert x.size >= 10_000_000
    fast, slow = gpu_ctx.div_a2_check(x, a)
    with np.errstate(all="ignore"):
        ref = x / (2.0 * a)
    ok_slow = _bits_equal(slow, ref)
    assert ok_slow.all(), f"device division differs from IEEE on {(~ok_slow).sum()} operands, e.g. x={x[~ok_slow][:3]}, a={a[~ok_slow][:3]}"
    ok = _bits_equal(fast, slow)
    assert ok.all(), f"div_a2 differs from the division on {(~ok).sum()} operands, e.g. x={x[~ok][:3]}, a={a[~ok][:3]}"
    # the window really was exercised on both sides
    ea2 = ((2.0 * a).view(np.uint64) >> np.uint64(52)) & np.uint64(0x7FF)
    ex = (x.view(np.uint64) >> np.uint64(52)) & np.uint64(0x7FF)
    inside = (ea2 >= 923) & (ea2 <= 1123) & (ex >= 123) & (ex <= 1622)
    assert inside.sum() > 5_000_000 and (~inside).sum() > 1_000_000


def test_sphere_sqrt_is_ieee_bit_for_bit(gpu_ctx):
    """The sphere test's square root (shapes.rs:67) as sphere_roots computes it:
    sqrt_win, the compiler's f64 sqrt sequence without its scaling of operands
    below 2^-767 (and its +-0 / +inf fixup), inside [2^-767, +inf), the full
    sqrt outside (trace_common.hpp).  Against the device's own
    sqrt and numpy's (IEEE) on > 10^7 operands: every exponent, both edges of
    the window and just outside, denormals, +-0, infinities, NaNs, negatives."""
    rng = np.random.default_rng(20261018)
    n = 1 << 21

    def f64(exp, size):
        mant = rng.integers(0, 1 << 52, size=size, dtype=np.uint64)
        e = np.broadcast_to(np.asarray(exp, dtype=np.uint64), (size,))
        return ((e << np.uint64(52)) | mant).view(np.float64)

    xs = [f64(rng.integers(1023 - 80, 1023 + 80, size=n), n),        # the renders' discriminants
          f64(rng.integers(0, 2047, size=2 * n), 2 * n)]              # every exponent, denormals included
    for e in range(252, 261):                                         # the window's lower edge 2^-767 (biased 256)
        xs.append(f64(e, n // 4))
    xs.append(f64(2046, n // 4))                                      # the largest finite binade
    # perfect squares and their neighbours (round-to-nearest ties do not exist for sqrt, but exact roots do)
    r = rng.uniform(1.0, 2.0 ** 26, n).astype(np.float64).round()
    sq = r * r
    xs += [sq, np.nextafter(sq, 0.0), np.nextafter(sq, np.inf)]
    xs.append(-np.abs(f64(rng.integers(0, 2047, size=n // 4), n // 4)))
    xs.append(np.array([0.0, -0.0, np.inf, -np.inf, np.nan, 5e-324, 2.0 ** -767, np.nextafter(2.0 ** -767, 0.0),
                        np.nextafter(2.0 ** -767, 1.0), 1.7976931348623157e308, 2.2250738585072014e-308, 1.0, 4.0]))
    x = np.concatenate(xs)
    assert x.size >= 10_000_000
    fast, slow = gpu_ctx.sqrt_check(x)
    with np.errstate(all="ignore"):
        ref = np.sqrt(x)
    ok_slow = _bits_equal(slow, ref)
    assert ok_slow.all(), f"device sqrt differs from IEEE on {(~ok_slow).sum()} operands, e.g. {x[~ok_slow][:3]}"
    ok = _bits_equal(fast, slow)
    assert ok.all(), f"sqrt_win differs from sqrt on {(~ok).sum()} operands, e.g. {x[~ok][:3]}"
    inside = (x >= 2.0 ** -767) & np.isfinite(x)
    assert inside.sum() > 5_000_000 and (~inside).sum() > 1_000_000
