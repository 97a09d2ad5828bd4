"""GPU parity of the gfx950 field arithmetic (ff.hpp, product-scanning Montgomery multiply
with hand-placed carry chains) against Python big ints, including the edge values that
stress carries (0, 1, p-1, all-ones words, values just below p)."""
import numpy as np
import pytest

import pyref as P

pytestmark = pytest.mark.gpu


def edge_values(mod, bits):
    vals = [0, 1, 2, mod - 1, mod - 2, (mod - 1) // 2, (mod + 1) // 2]
    vals += [(1 << k) % mod for k in (31, 32, 63, 64, 127, 128, 191, 192, 254, bits - 1)]
    vals += [((1 << (32 * j)) - 1) % mod for j in range(1, (bits + 31) // 32)]
    return vals


def random_values(mod, bits, n, seed):
    rng = np.random.default_rng(seed)
    out = []
    while len(out) < n:
        v = int.from_bytes(rng.bytes((bits + 7) // 8), "little") & ((1 << bits) - 1)
        if v < mod:
            out.append(v)
    return out


@pytest.mark.parametrize("field", ["fr", "fp"])
def test_field_ops_vs_bigint(gpu_ctx, field):
    mod, bits, words, R = ((P.R_MOD, 255, 4, 1 << 256) if field == "fr"
                           else (P.P_MOD, 381, 6, 1 << 384))
    e = edge_values(mod, bits)
    xs = e * len(e) + random_values(mod, bits, 4000, 1)
    ys = [v for v in e for _ in e] + random_values(mod, bits, 4000, 2)
    to_mont = lambda v: v * R % mod  # noqa: E731
    from_mont = lambda v: v * pow(R, -1, mod) % mod  # noqa: E731
    enc = lambda vals: np.array([P.int_to_limbs(to_mont(v), words) for v in vals],  # noqa: E731
                                dtype=np.uint64)
    dec = lambda arr: [from_mont(P.limbs_to_int(r)) for r in arr]  # noqa: E731
    A, B = enc(xs), enc(ys)
    assert dec(gpu_ctx.field_op(field, "mul", A, B)) == [x * y % mod for x, y in zip(xs, ys)]
    assert dec(gpu_ctx.field_op(field, "add", A, B)) == [(x + y) % mod for x, y in zip(xs, ys)]
    assert dec(gpu_ctx.field_op(field, "sub", A, B)) == [(x - y) % mod for x, y in zip(xs, ys)]
    assert dec(gpu_ctx.field_op(field, "sqr", A)) == [x * x % mod for x in xs]
    k = 300
    inv = dec(gpu_ctx.field_op(field, "inv", A[-k:]))
    assert inv == [pow(x, -1, mod) if x else 0 for x in xs[-k:]]
    # outputs are canonical (fully reduced) limbs
    out = gpu_ctx.field_op(field, "mul", A, B)
    assert all(P.limbs_to_int(r) < mod for r in out)
